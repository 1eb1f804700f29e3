"""Model families: motion LSTM/GRU classifier, char-level LM, bidirectional stacks."""
from .motion import MotionModel  # noqa: F401
from .rnn import GRU, LSTM  # noqa: F401
