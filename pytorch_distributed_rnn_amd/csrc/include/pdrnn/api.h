// C ABI between the hipcc-compiled kernels (csrc/kernels/*.hip) and the
// g++-compiled host runtime / torch bindings (csrc/bindings.cpp).
//
// Every launcher takes plain pointers plus a hipStream_t and returns the HIP
// error of the launch.  Argument structs are POD so that both compilers agree
// on their layout.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDRNN_MAX_LAYERS 4

// ----------------------------------------------------------------------------
// Fused small-hidden LSTM stack (H <= 64, input size <= H): every layer of the
// stack runs inside ONE launch, layer l working on timestep t-l while layer 0
// works on t (wavefront pipeline); one workgroup owns NB sequences for all T.
// ----------------------------------------------------------------------------
typedef struct {
  const float* x;            // input, element (b,t,i) at b*x_sb + t*x_st + i
  const int64_t* idx;        // optional gather: batch row b reads x sequence idx[b]
  int64_t x_sb, x_st;
  const float* w_ih[PDRNN_MAX_LAYERS];  // [4H, I_l]   gate order i,f,g,o
  const float* w_hh[PDRNN_MAX_LAYERS];  // [4H, H]
  const float* b_ih[PDRNN_MAX_LAYERS];  // [4H] or NULL
  const float* b_hh[PDRNN_MAX_LAYERS];  // [4H] or NULL
  const float* h0;           // [NL, B, H] or NULL (zeros)
  const float* c0;           // [NL, B, H] or NULL
  float* hseq;               // training: [NL, B, T, H] every layer's h_t
  float* act;                // training: [NL, B, T, 5, H] post-activation i,f,g,o and c_t
  float* out;                // inference: top-layer output (may be NULL), (b,t,j) at b*o_sb+t*o_st+j
  int64_t o_sb, o_st;
  float* hn;                 // [NL, B, H]
  float* cn;                 // [NL, B, H]
  uint64_t* stamps;          // diagnostics: [grid, 4] s_memtime/s_memrealtime around the loop, or NULL
  // ---- fused classifier head + softmax cross-entropy (train step fusion) ----
  // When head_w != NULL (requires nb == 1, save == 1): after the last step the
  // top layer's h_T feeds logits = head_w h_T + head_b, the per-sequence CE
  // loss against labels[idx[b]] (mean over B: scaled by inv_batch), and
  // writes into slab row b: dW_head, db_head (cols head_off_w / head_off_b)
  // and [loss, correct] (cols stat_off); dL/dh_T goes to dh_top [B, H].
  const float* head_w;       // [C, H]
  const float* head_b;       // [C] or NULL
  const int64_t* labels;     // [N] class ids (indexed through idx when given)
  float* slab;               // [B, P] (shared with the backward's slab)
  float* dh_top;             // [B, H]
  int64_t slab_P, head_off_w, head_off_b, stat_off;
  float inv_batch;
  int C;
  int B, T, I, NL;
  int cell;                  // 0 = LSTM, 1 = GRU (packed as a 4-row-block stack, see ops/gru.py)
  int x_bf16;                // x holds bf16 values (read once into LDS; requires the LDS-resident x path)
  int prio;                  // lower the waves' issue priority as the recurrence progresses (see prio_by_progress)
  int w_bf16;                // round the fp32 W_ih / W_hh to bf16 as they are loaded (bf16 models: no cast pass)
  // sequence-in-wave forward (lstm_sw.hip): the staged, widened layer-0 input
  // rows [B*T][xg_ld] for the deferred-dW kernel (NULL: not written)
  float* xg_out;
  int xg_ld;
  // sequence-in-wave mode 5 with stamps: the phase-stamped build (stamps rows
  // of 24: the loop stamps, then per-step cycle sums of waves 0 / 2)
  int phase_stamps;
} PdrnnLstmSmallFwdArgs;

typedef struct {
  const float* x;
  const int64_t* idx;
  int64_t x_sb, x_st;
  const float* w_ih[PDRNN_MAX_LAYERS];
  const float* w_hh[PDRNN_MAX_LAYERS];
  const float* h0;
  const float* c0;
  const float* hseq;         // saved by the forward
  const float* act;          // saved by the forward
  const float* dout;         // grad of top-layer output, (b,t,j) at b*d_sb+t*d_st+j; NULL = 0
  int64_t d_sb, d_st;
  const float* dhn;          // [NL,B,H] or NULL
  const float* dcn;          // [NL,B,H] or NULL
  float* dx;                 // (b,t,i) at b*dx_sb+t*dx_st+i, or NULL (input grad not needed)
  int64_t dx_sb, dx_st;
  float* dh0;                // [NL,B,H] or NULL
  float* dc0;                // [NL,B,H] or NULL
  float* slab;               // [grid, P] per-workgroup partial parameter gradients
  int64_t P;
  int64_t off_wih[PDRNN_MAX_LAYERS], off_whh[PDRNN_MAX_LAYERS];
  int64_t off_bih[PDRNN_MAX_LAYERS], off_bhh[PDRNN_MAX_LAYERS];  // -1 = no bias
  uint64_t* stamps;          // diagnostics (see forward), or NULL
  int dhn_top_only;          // dhn is [B, H] for the top layer only (fused head path)
  int B, T, I, NL;
  int cell;                  // 0 = LSTM, 1 = GRU (packed as a 4-row-block stack, see ops/gru.py)
  int x_bf16;                // x holds bf16 values (read once into LDS; requires the LDS-resident x path)
  // Deferred weight gradients (pdrnn_lstm_small_bwd_dwout): the recurrence
  // keeps no dW accumulators and writes the pre-activation gate gradients of
  // (layer l, row b, step t) to dg_out + ((l*B + b)*T + t)*dg_st + [0, 4H)
  // instead (dg_out may be `act` itself, dg_st = 5H: each lane overwrites the
  // activation slot it has just consumed); pdrnn_lstm_small_dw then forms
  // dW_ih, dW_hh and the biases on the matrix cores.  dg_out must have
  // PDRNN_DW_PAD_ROWS padding rows behind the last layer (the kernel zeroes them).
  float* dg_out;
  int64_t dg_st;
  float* xg_out;             // DWOUT: [B*T][xg_ld] fp32 copy of the (gathered, widened) layer-0 input
  int xg_ld;
  int prio;                  // see the forward
  int w_bf16;                // see the forward
} PdrnnLstmSmallBwdArgs;

// Weight gradients of the small-H stack from saved gate gradients, on the
// fp32 matrix cores (lstm_small_dw.hip): for every layer l,
//   dW_ih[l] = sum_{b,t} dg[l,b,t]^T in[l,b,t]     (in = x for l = 0, else h^{l-1}_t)
//   dW_hh[l] = sum_{b,t} dg[l,b,t]^T h^l_{t-1}      (h_{-1} = 0)
//   db[l]    = sum_{b,t} dg[l,b,t]                  (written to both bias slots)
// split over `chunks` contiguous (b, t) row ranges: chunk c writes slab row c
// (columns in the stack's flat parameter layout), reduced afterwards by
// pdrnn_slab_reduce_adam.
// Padding contract (the kernel streams whole stages of up to
// PDRNN_DW_PAD_ROWS rows without clamps): hseq readable from row -1 of layer
// 0 (H floats before it) through PDRNN_DW_PAD_ROWS rows past the last layer;
// dg and xg readable through PDRNN_DW_PAD_ROWS rows past their end (dg: those
// rows finite -- the BPTT zeroes them).
#define PDRNN_DW_PAD_ROWS 32
typedef struct {
  const float* xg;           // layer-0 input rows [B*T][xg_ld] fp32 (the BPTT's xg_out), xg_ld = I rounded up to 4
  int xg_ld;
  const float* hseq;         // [NL, B, T, H] saved by the forward
  const float* dg;           // gate gradients, (l,b,t) row at ((l*B+b)*T+t)*dg_st
  int64_t dg_st;
  float* slab;               // [chunks, P]
  int64_t P;
  int64_t off_wih[PDRNN_MAX_LAYERS], off_whh[PDRNN_MAX_LAYERS];
  int64_t off_bih[PDRNN_MAX_LAYERS], off_bhh[PDRNN_MAX_LAYERS];
  int B, T, I, NL, chunks;
} PdrnnLstmSmallDwArgs;
// 1 when the deferred-dW backward covers (H, NL, T) (H in {16, 32, 64}, T >= 4)
int pdrnn_lstm_small_dwout_ok(int H, int NL, int T);
// default chunk count (= slab rows) for a B x T batch
int pdrnn_lstm_small_dw_chunks(int H, int NL, int B, int T);
hipError_t pdrnn_lstm_small_dw(const PdrnnLstmSmallDwArgs* a, int H, hipStream_t stream);
// BPTT of the lean fused-step contract with the weight gradients deferred to
// pdrnn_lstm_small_dw (a->dg_out set, a->slab unused); grid <= 0: persistent
// grid of the resident capacity (query with pdrnn_lstm_small_bwd_dwout_grid);
// nb = sequences per workgroup (1 or 2: pdrnn_lstm_small_bwd_dwout_nb).
hipError_t pdrnn_lstm_small_bwd_dwout(const PdrnnLstmSmallBwdArgs* a, int H, int grid, int nb, hipStream_t stream);
int pdrnn_lstm_small_bwd_dwout_nb(int H, int NL, int T, int B);
int pdrnn_lstm_small_bwd_dwout_grid(int H, int NL, int T, int B, int nb);

// Query the launch geometry chosen for (H, B): returns grid size (number of slab rows).
int pdrnn_lstm_small_grid(int H, int B, int nb);
int pdrnn_lstm_small_supported(int H, int I, int NL);
int pdrnn_lstm_small_max_split(int H, int NL, int backward);
// split = lanes per hidden unit (forward S in {2,4,8}; backward S2 in {2,4})
hipError_t pdrnn_lstm_small_fwd(const PdrnnLstmSmallFwdArgs* a, int H, int nb, int split, int save,
                                hipStream_t stream);
// grid <= 0: natural grid (persistent for the unit-group map); query with _bwd_grid
hipError_t pdrnn_lstm_small_bwd(const PdrnnLstmSmallBwdArgs* a, int H, int nb, int split, int grid,
                                hipStream_t stream);
int pdrnn_lstm_small_bwd_grid(int H, int NL, int T, int B, int nb, int split);
// One-launch training step of the latency regime: forward + head/CE epilogue
// + BPTT of sequence b in workgroup b (lean backward contract, gridb == B).
int pdrnn_lstm_small_step_ok(int H, int NL, int B, int nb_fwd, int split_fwd, int nb_bwd, int split_bwd,
                             int gridb);
hipError_t pdrnn_lstm_small_step(const PdrnnLstmSmallFwdArgs* f, const PdrnnLstmSmallBwdArgs* b, int H,
                                 hipStream_t stream);

// ----------------------------------------------------------------------------
// Sequence-in-wave LSTM / GRU stack (kernels/lstm_sw.hip): H = 32, 1 or 2
// layers, input size <= 12, lean training contract (zero initial state, loss
// through the fused head on h_T; the GRU as the packed 4-block stack, cell = 1).  A sequence's whole recurrence lives in ONE wave
// (mode 0: one sequence per wave, mode 1: two), or in one wave per layer of a
// 2-layer stack (mode 2), so h_t never crosses a workgroup barrier inside a
// layer.  The forward writes act / hseq / xg_out like the gate-split forward
// plus the head's slab rows; the backward writes the gate gradients over the
// activations (dg_out = act, dg_st = 5H) for pdrnn_lstm_small_dw.
// ----------------------------------------------------------------------------
int pdrnn_lstm_sw_ok(int H, int I, int NL, int cell);
int pdrnn_lstm_sw_fits(int NL, int B, int T);
// sequences per wave (and per workgroup) of a sequence-in-wave mode
int pdrnn_lstm_sw_nb(int mode);
// mode for a batch of B sequences (PDRNN_TUNE sw_mode / sw_bwd_mode override)
int pdrnn_lstm_sw_mode(int NL, int B, int backward);
hipError_t pdrnn_lstm_sw_fwd(const PdrnnLstmSmallFwdArgs* a, int mode, hipStream_t stream);
hipError_t pdrnn_lstm_sw_bwd(const PdrnnLstmSmallBwdArgs* a, int mode, hipStream_t stream);

// Column sums of a [rows, P] fp32 slab into out[P] (out = beta*out + sum).
// Two deterministic passes through `work` ([split, P] floats, split <= 64).
hipError_t pdrnn_slab_reduce(const float* slab, int64_t rows, int64_t P, float* out, float beta,
                             float* work, int split, hipStream_t stream);
// Two slabs reduced side by side (columns of A then of B); the first n_out
// summed columns go to out, the rest to out_tail.
hipError_t pdrnn_slab2_reduce(const float* A, int64_t rowsA, int64_t PA, const float* Bs, int64_t rowsB, int64_t PB,
                              int64_t n_out, float* out, float* out_tail, float* work, int split, const int* colmap,
                              int64_t ldA, hipStream_t stream);
// First pass only (work[split][PA+PB] partial column sums); the second pass
// can be fused into its consumer (pdrnn_adam_partials).
// colmap (optional, with ldA = A's leading dimension): output column p < PA
// reads A column colmap[p] (GRU packed layout -> nn.GRU order); NULL = identity
hipError_t pdrnn_slab2_reduce_pass1(const float* A, int64_t rowsA, int64_t PA, const float* Bs, int64_t rowsB,
                                   int64_t PB, float* work, int split, const int* colmap, int64_t ldA,
                                   hipStream_t stream);
// Same, with columns [P_a, P) written to out_b instead (e.g. loss statistics).
hipError_t pdrnn_slab_reduce2(const float* slab, int64_t rows, int64_t P, int64_t P_a, float* out_a,
                              float* out_b, float* work, int split, hipStream_t stream);

// ----------------------------------------------------------------------------
// Fused cross-entropy (+ accuracy): mean loss over valid rows, dlogits saved.
// ----------------------------------------------------------------------------
typedef struct {
  const void* logits;        // [N, C] fp32/bf16/fp16 (row stride ld)
  int64_t ld;
  int dtype;                 // 0 fp32, 1 bf16, 2 fp16
  const int64_t* labels;     // [N]
  int64_t N, C;
  int64_t ignore_index;
  float* row_loss;           // [N] scratch
  float* dlogits;            // [N, C] fp32 (softmax - onehot) / n_valid, or NULL
  float* partial;            // [nblocks, 3]  (loss sum, n_valid, n_correct)
  float* out;                // [3] loss mean, n_valid, n_correct
} PdrnnXentArgs;
hipError_t pdrnn_xent_fwd(const PdrnnXentArgs* a, hipStream_t stream);
int pdrnn_xent_partial_blocks(int64_t N, int64_t C);
// dst = dlogits * (grad_out[0] / stats[1])   (stats = PdrnnXentArgs.out)
hipError_t pdrnn_xent_bwd(const float* dlogits, const float* grad_out, const float* stats, void* dst,
                          int64_t n, int out_dtype, hipStream_t stream);

// ----------------------------------------------------------------------------
// Tuning overrides (runtime/tune.cpp): PDRNN_TUNE="key=value,...".  _str
// copies the value of `key` into out (NUL-terminated) and returns 1 when the
// key is present; _int returns its integer value, or dflt when absent / not
// an integer.
// ----------------------------------------------------------------------------
int pdrnn_tune_str(const char* key, char* out, int out_len);
int pdrnn_tune_int(const char* key, int dflt);

// ----------------------------------------------------------------------------
// Fused Adam / AdamW over flat fp32 buffers (torch.optim.Adam semantics).
// ----------------------------------------------------------------------------
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* max_exp_avg_sq;     // amsgrad only, else NULL
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay;
  float bias_correction1, bias_correction2_sqrt;
  float grad_scale;          // multiply grads (e.g. 1/world for a sum all-reduce)
  int decoupled;             // AdamW
  int maximize;
  const float* lr_ptr;       // optional device lr (graph-capturable); overrides lr
  const float* step_ptr;     // optional device step count for bias correction (capturable)
  // optional: advance the device step count in-kernel (graph replay needs no
  // separate increment launch): the step used is *step_advance + 1, written
  // back by the last workgroup to finish (arrival ticket, reset to 0 after)
  float* step_advance;
  unsigned int* ticket;
  // != nullptr and nonzero at run time: the launch returns without touching
  // anything (a step whose results are invalid, decided on the device)
  const int* skip;
} PdrnnAdamArgs;
hipError_t pdrnn_adam_flat(const PdrnnAdamArgs* a, hipStream_t stream);

// One launch per training step in the latency regime (two layers, B <= two
// workgroups per CU, T % 4 == 0): forward mode 5 + head/CE, then BPTT mode 4
// with its matrix-core dW waves (kernels/lstm_sw.hip lstm_sw_step_kernel).
int pdrnn_lstm_sw_step_ok(int NL, int B, int T);
hipError_t pdrnn_lstm_sw_step(const PdrnnLstmSmallFwdArgs* f, const PdrnnLstmSmallBwdArgs* b, hipStream_t stream);
// g *= min(1, max_norm / (||g|| + eps)) with no host sync; work: [nparts]
// floats (nparts <= 1024 partial sums of squares), out: [2] = (scale, norm).
hipError_t pdrnn_clip_flat(float* g, int64_t n, float max_norm, float eps, float* work, int nparts, float* out,
                           hipStream_t stream);

// ----------------------------------------------------------------------------
// Embedding gather / deterministic CSR backward (perm = stable argsort of idx,
// offsets[v] = first position of vocabulary row v in the sorted order).
// ----------------------------------------------------------------------------
hipError_t pdrnn_embedding_fwd(const float* weight, const int64_t* idx, float* out, int64_t n_idx,
                               int64_t dim, int64_t num_embeddings, hipStream_t stream);
hipError_t pdrnn_embedding_fwd16(const float* weight, const int64_t* idx, uint16_t* out, int64_t n_idx, int64_t dim,
                                 int64_t num_embeddings, int dtype, hipStream_t stream);
// dout_dtype: 0 bf16, 1 fp16, 2 fp32
// Small-vocabulary form: each row's contribution list split into `pieces`
// equal parts (partials: [V][pieces][dim] fp32 scratch), summed in order.
// Stable in-tree sort of n indices by row (V <= 16384): perm [n], offsets
// [V + 1] (int64), scratch int32 [pdrnn_embedding_sort_scratch(n, V)].
int64_t pdrnn_embedding_sort_scratch(int64_t n, int64_t V);
hipError_t pdrnn_embedding_sort(const int64_t* idx, int64_t n, int64_t V, int* scratch, int64_t* perm,
                                int64_t* offsets, hipStream_t stream);
// accumulate: dweight += the row sums instead of dweight = (a gradient buffer)
hipError_t pdrnn_embedding_bwd_pieces(const void* dout, int dout_dtype, const int64_t* perm, const int64_t* offsets,
                                     float* partials, int pieces, float* dweight, int64_t num_embeddings, int64_t dim,
                                     int64_t padding_idx, int accumulate, hipStream_t stream);
hipError_t pdrnn_embedding_bwd_csr2(const void* dout, int dout_dtype, const int64_t* perm, const int64_t* offsets,
                                   float* dweight, int64_t num_embeddings, int64_t dim, int64_t padding_idx,
                                   hipStream_t stream);
hipError_t pdrnn_embedding_bwd_csr(const float* dout, const int64_t* perm, const int64_t* offsets,
                                   float* dweight, int64_t num_embeddings, int64_t dim,
                                   int64_t padding_idx, hipStream_t stream);

// ---- large-H LSTM (MFMA per-step kernels; bf16 / fp16 / fp32 storage) ------
// Storage pointers are void*: elements of the dtype passed to the launchers
// (0 bf16, 1 fp16, 2 fp32).
// One direction of a layer.  Gate-interleaved layouts: column / row 4u+q is
// gate q (i, f, g, o) of unit u.
typedef struct {
  const void* w;           // [4H, H] W_hh, gate-interleaved rows (forward GEMM: h Wp^T)
  const void* wt;          // [H, 4H] W_hh^T, torch gate-blocked order (backward GEMM: dgates W_hh)
  const void* xp;          // input projection incl. bias, [t, b, col] at t*xp_st + b*xp_sb + col
  int64_t xp_sb, xp_st;
  const void* h0;          // [B, H] or null
  const float* c0;         // [B, H] or null
  void* hseq;              // outputs h_t at t*hseq_st + b*hseq_sb + u
  int64_t hseq_sb, hseq_st;
  float* cseq;             // [T, B, H] fp32 cell states
  void* acts;              // [T, B, 4H] activated gates
  void* dgates;            // [T, B, 4H] pre-activation gate gradients, gate-blocked (i|f|g|o)
  const void* dout;        // grad of hseq (same strides as dout_sb / dout_st) or null
  int64_t dout_sb, dout_st;
  const float* dhn;        // [B, H] or null
  const float* dcn;        // [B, H] or null
  float* dc_carry;         // [B, H] fp32 scratch
  float* dh0;              // [B, H] or null
  float* dc0;              // [B, H] or null
} PdrnnLstmLargeDir;

typedef struct {
  PdrnnLstmLargeDir dir[2];
  int B, H, T;
  int step;                // processing-order step index (forward) / backward step index
  int reverse_mask;        // bit d set: direction d runs time-reversed
  int splitk;              // backward: K slices (> 1 needs ws)
  int splitk_big;          // split-K tile: 0 = 32x32, 1 = 128x128
  int bwd_pp;              // backward: ping-pong GEMM into ws, then the cell kernel (needs ws, splitk = 1)
  int cell;                // 0 = LSTM; 1 = GRU packed as [r|z|n_x|n_h] (cseq = fp32 h, acts = r,z,n,n_h)
  float* ws;               // backward split-K partials [splitk][2][B][H] fp32
  // persistent kernels: processing-order steps [s0, s1) of the T-step layer
  // (s1 = 0: all of them).  A range after the first resumes from the state the
  // earlier range left in hseq / cseq (forward) or dgates / dc_carry
  // (backward); the sync counters carry over (zeroed before the first range).
  int s0, s1;
} PdrnnLstmLargeStepArgs;

int pdrnn_lstm_large_supported(int H);
int pdrnn_lstm_large_bwd_splitk(int B, int H, int ndir, int* big);
// 1: run the backward step as the ping-pong GEMM (fp32 dh into ws) + the cell kernel
int pdrnn_lstm_large_bwd_pp(int B, int H, int ndir, int dtype);
// dtype 0 = bf16, 1 = fp16, 2 = fp32; tile -1 = auto, 0..3 = 32x64 / 64x64 / 128x128 / 256x128 block tiles
hipError_t pdrnn_lstm_large_step(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, int dtype, int tile,
                                 hipStream_t stream);
hipError_t pdrnn_lstm_large_bwd_first(const PdrnnLstmLargeStepArgs* a, int ndir, int dtype, hipStream_t stream);
// Row-owning fp32 recurrence (kernels/lstm_rows_f32.hip): one launch per layer
// pass, 16 batch rows and all of W_hh per workgroup, no grid sync; H = 128,
// fp32 storage.  The backward needs pdrnn_lstm_large_bwd_first first.
int pdrnn_lstm_rows_f32_supported(int H, int dtype);
hipError_t pdrnn_lstm_rows_f32(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, hipStream_t stream);
// Persistent recurrence: all T steps of a layer in one launch (occupancy-checked, all workgroups co-resident) with
// W_hh register-resident.  persist_mt: rows-per-workgroup / 16 for this shape
// (0 = not covered); counters: ndir * ceil(B / (16 mt)) zeroed ints; err: an
// int set to 1 if a grid-sync spin timed out (sticky, if not null: also set,
// never cleared); mode: 0 (diagnostic bits, see the kernel); xchg: null, or for a
// 16-bit forward nslots (>= 2) * ndir * B * H zeroed dwords (16-byte aligned): the tagged
// h exchange instead of the arrival counters (lstm_large.hip ps_poll_h).
// Weight-shadow pack (kernels/shadow_pack.hip): up to PDRNN_PACK_MAX_JOBS
// 3-D strided gathers dst[i0,i1,i2] = src[...] (+ src2[...]) from bf16 /
// fp16 / fp32 sources (sdtype), converted to dtype, one launch.  Strides
// in elements; tile0 is filled in by pdrnn_shadow_pack.
#define PDRNN_PACK_MAX_JOBS 16
typedef struct PdrnnPackJob {
  const void* src;
  const void* src2;  // optional second addend (same strides and dtype), or null
  void* dst;
  int64_t ss[3];
  int64_t ds[3];
  int n[3];
  int dtype;   // destination: 0 bf16, 1 fp16, 2 fp32
  int sdtype;  // sources: same codes
  int vec;     // set by pdrnn_shadow_pack: the 4-wide path applies
  int64_t tile0;
} PdrnnPackJob;
typedef struct PdrnnPackBatch {
  PdrnnPackJob job[PDRNN_PACK_MAX_JOBS];
  int njobs;
} PdrnnPackBatch;
int64_t pdrnn_shadow_pack_tiles(const PdrnnPackJob* j);
hipError_t pdrnn_shadow_pack(PdrnnPackBatch* b, hipStream_t stream);
int pdrnn_lstm_large_persist_mt(int B, int H, int ndir, int dtype, int cus);
hipError_t pdrnn_lstm_large_persist(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, int dtype, int mt,
                                    int* counters, int* err, int* sticky, int mode, uint32_t* xchg,
                                    int nslots, hipStream_t stream);
// Time-batched GEMM of the large-H layers (kernels/gemm.hip), 16-bit inputs:
//   C[M, N] (= or +=) sum over the K segments of op(A) op(B) (+ bias[n])
// A: a_kmajor ? element (m, k) at A[k * lda + m] : A[m * lda + k]
// B: b_kmajor ? element (n, k) at B[k * ldb + n] : B[n * ldb + k]
// segment 2 (K2 > 0): A2 / B2 with lda2 / ldb2, same layouts.
// C: fp32 (accumulate: C += ...) or, with c_16bit, the input dtype (+ fp32 bias).
typedef struct {
  const void* A;
  const void* B;
  const void* A2;
  const void* B2;
  void* C;
  const float* bias;
  int64_t lda, ldb, lda2, ldb2, ldc;
  int M, N, K, K2;
  int dtype;  // 0 bf16, 1 fp16
  int a_kmajor, b_kmajor, c_16bit, accumulate;
  int splitk;              // > 1: K split over blockIdx.y, partial s at C + s * c_split_stride (fp32)
  int64_t c_split_stride;
  int variant;             // schedule variant (tuning)
} PdrnnGemmArgs;
int pdrnn_gemm_supported(const PdrnnGemmArgs* a);
// schedule variants compiled into this build (first = default)
int pdrnn_gemm_variants(int* out, int max);
hipError_t pdrnn_gemm(const PdrnnGemmArgs* a, hipStream_t stream);
// tile: -1 auto, 0..3 = 32x64 / 64x64 / 128x128 / 256x128 block tiles
hipError_t pdrnn_gemm_nt(const void* A, int64_t lda, const void* Bt, int64_t ldb, float* C, int64_t ldc,
                         int M, int N, int K, int dtype, int tile, hipStream_t stream);

// fp32-product GEMM on the matrix cores (kernels/gemm_f32.hip): fp32 or
// 16-bit inputs (widened exactly), any of the four operand layouts, optional
// second K segment, fp32 bias, row sums of op(A) over K (bias gradients), split-K.
typedef struct {
  const void* A;
  const void* B;
  const void* A2;
  const void* B2;
  void* C;
  const float* bias;         // [N], added in the epilogue (not with split-K)
  float* rowsum;             // optional [splitk][M]: sum over K of op(A)(m, k)
  int64_t lda, ldb, lda2, ldb2, ldc;
  int M, N, K, K2;
  int in_dtype;              // 0 bf16, 1 fp16, 2 fp32 (A, B, A2, B2)
  int out_dtype;             // 2 fp32, else the 16-bit input dtype
  int a_kmajor, b_kmajor, accumulate;
  int splitk;                // > 1: fp32 partials at C + s * c_split_stride (ldc = N)
  int64_t c_split_stride;
  int vec;                   // every row stride a multiple of 4 elements and every base 16-byte aligned
} PdrnnGemmF32Args;
int pdrnn_gemm_f32_supported(const PdrnnGemmF32Args* a);
hipError_t pdrnn_gemm_f32(const PdrnnGemmF32Args* a, hipStream_t stream);
// out[i] (= or +=) sum_s part[s * n + i] in a fixed order
hipError_t pdrnn_splitk_sum(const float* part, int splitk, int64_t n, float* out, int accumulate, hipStream_t stream);
// column sums of X [rows, cols] (row stride ld, dtype 0 bf16 / 1 fp16 / 2 fp32):
// partials part[groups][cols], then pdrnn_splitk_sum(part, groups, cols, out)
int pdrnn_col_sum_groups(int64_t rows, int64_t cols);
hipError_t pdrnn_col_sum(const void* X, int dtype, int64_t rows, int64_t cols, int64_t ld, float* part, int groups,
                         hipStream_t stream);

// Adam whose gradient is the fixed-order sum of `split` rows of work[split][P_total]
// (columns [0, a->n)); grad_out receives it, columns [n, n + n_stats) -> stats_out.
hipError_t pdrnn_adam_partials(const PdrnnAdamArgs* a, const float* work, int split, int64_t P_total,
                               float* grad_out, float* stats_out, int n_stats, hipStream_t stream);
// One-pass reduction of the fused step's [rowsA, ldA] (through colmap) and
// [rowsB, PB] gradient slabs into grad_out[0:n_out] (+ tail_out for the
// columns past n_out), with the Adam step of each element when a != nullptr.
// slot_step != NULL: tail_out is a [ring_rows, tail] ring and the tail goes to
// row ((int)*slot_step + slot_offset) mod ring_rows (graph-replayed steps).
hipError_t pdrnn_slab_reduce_adam(const PdrnnAdamArgs* a, const float* A, int64_t rowsA, int64_t PA, int64_t ldA,
                                  const int* colmap, const float* Bs, int64_t rowsB, int64_t PB, int64_t n_out,
                                  float* grad_out, float* tail_out, const float* slot_step, int slot_offset,
                                  int ring_rows, hipStream_t stream);

// Diagnostics: a single wave that spins for `microseconds` (bounded, <= 60 s).
// Communicator-watchdog tests only.
hipError_t pdrnn_debug_spin(uint64_t microseconds, hipStream_t stream);
// Diagnostics: `workgroups` x `threads` spinning for `microseconds` each
// (bounded, <= 10 s), `lds_bytes` of LDS apiece (CU occupancy).
hipError_t pdrnn_debug_spin_cus(uint64_t microseconds, int workgroups, int threads, int lds_bytes,
                                hipStream_t stream);

#ifdef __cplusplus
}
#endif
