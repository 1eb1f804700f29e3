// Stand-alone probe of the sequence-in-wave LSTM kernels (csrc/kernels/lstm_sw.hip)
// against an fp64 CPU reference, and an A/B timing against the gate-split /
// K-split kernels of lstm_small.hip on the same buffers.  No torch: builds in
// seconds and runs on a fresh GPU box without the torch import.
//
//   bench/sw_probe.sh            (build + run: B=180 and 1440, every mode)
//   sw_probe B [reps] [modes...]  mode 0-3, 6 = sequence-in-wave (lstm_sw.hip),
//                                 9 = lstm_small (gate-split / K-split family)
//   (mode 7, the bf16 matrix-core recurrence lstm_mb.hip, was removed in round 6:
//   1.2-3.3x slower than these fp32 VALU kernels, docs/DESIGN.md §2b)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pdrnn/api.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

static const int H = 32, I = 9, C = 6;

struct Ref {
  std::vector<double> act;   // [NL][B][T][5H]
  std::vector<double> hseq;  // [NL][B][T][H]
  std::vector<double> dhtop; // [B][H]
  std::vector<double> dz;    // [NL][B][T][4H]
};

static double sg(double z) { return 1.0 / (1.0 + std::exp(-z)); }

static void reference(int NL, int B, int T, const std::vector<float>& x, const std::vector<int64_t>& idx,
                      const std::vector<int64_t>& lab, std::vector<float>* wih, std::vector<float>* whh,
                      std::vector<float>* bih, std::vector<float>* bhh, const std::vector<float>& hw,
                      const std::vector<float>& hb, Ref& R) {
  R.act.assign((size_t)NL * B * T * 5 * H, 0.0);
  R.hseq.assign((size_t)NL * B * T * H, 0.0);
  R.dhtop.assign((size_t)B * H, 0.0);
  R.dz.assign((size_t)NL * B * T * 4 * H, 0.0);
  for (int b = 0; b < B; ++b) {
    const float* xb = x.data() + (size_t)idx[b] * T * I;
    for (int l = 0; l < NL; ++l) {
      const int Iin = l == 0 ? I : H;
      std::vector<double> h(H, 0.0), c(H, 0.0);
      for (int t = 0; t < T; ++t) {
        std::vector<double> in(Iin);
        for (int k = 0; k < Iin; ++k)
          in[k] = l == 0 ? xb[t * I + k] : R.hseq[(((size_t)(l - 1) * B + b) * T + t) * H + k];
        double z[4 * H];
        for (int r = 0; r < 4 * H; ++r) {
          double s = (double)bih[l][r] + bhh[l][r];
          for (int k = 0; k < Iin; ++k) s += (double)wih[l][r * Iin + k] * in[k];
          for (int k = 0; k < H; ++k) s += (double)whh[l][r * H + k] * h[k];
          z[r] = s;
        }
        double* a = &R.act[(((size_t)l * B + b) * T + t) * 5 * H];
        for (int u = 0; u < H; ++u) {
          const double ig = sg(z[u]), fg = sg(z[H + u]), gg = std::tanh(z[2 * H + u]), og = sg(z[3 * H + u]);
          c[u] = fg * c[u] + ig * gg;
          h[u] = og * std::tanh(c[u]);
          a[u] = ig; a[H + u] = fg; a[2 * H + u] = gg; a[3 * H + u] = og; a[4 * H + u] = c[u];
          R.hseq[(((size_t)l * B + b) * T + t) * H + u] = h[u];
        }
      }
    }
    // head + CE
    const double* hT = &R.hseq[(((size_t)(NL - 1) * B + b) * T + T - 1) * H];
    double lg[C], m = -1e300;
    for (int cc = 0; cc < C; ++cc) {
      double s = hb[cc];
      for (int u = 0; u < H; ++u) s += (double)hw[cc * H + u] * hT[u];
      lg[cc] = s;
      m = std::max(m, s);
    }
    double se = 0;
    for (int cc = 0; cc < C; ++cc) se += std::exp(lg[cc] - m);
    for (int u = 0; u < H; ++u) {
      double d = 0;
      for (int cc = 0; cc < C; ++cc)
        d += hw[cc * H + u] * ((std::exp(lg[cc] - m) / se - (cc == lab[idx[b]] ? 1.0 : 0.0)) / B);
      R.dhtop[(size_t)b * H + u] = d;
    }
    // BPTT
    std::vector<double> dh_in((size_t)T * H, 0.0);  // dh from the layer above, per step
    for (int l = NL - 1; l >= 0; --l) {
      const int Iin = l == 0 ? I : H;
      std::vector<double> dh(H, 0.0), dc(H, 0.0), dxn((size_t)T * H, 0.0);
      for (int t = T - 1; t >= 0; --t) {
        const double* a = &R.act[(((size_t)l * B + b) * T + t) * 5 * H];
        double dzv[4 * H];
        for (int u = 0; u < H; ++u) {
          double dht = dh[u] + dh_in[(size_t)t * H + u];
          if (l == NL - 1 && t == T - 1) dht += R.dhtop[(size_t)b * H + u];
          const double ig = a[u], fg = a[H + u], gg = a[2 * H + u], og = a[3 * H + u], ct = a[4 * H + u];
          const double cp = t > 0 ? R.act[(((size_t)l * B + b) * T + t - 1) * 5 * H + 4 * H + u] : 0.0;
          const double tc = std::tanh(ct);
          const double dcp = dc[u] + dht * og * (1 - tc * tc);
          dzv[u] = dcp * gg * ig * (1 - ig);
          dzv[H + u] = dcp * cp * fg * (1 - fg);
          dzv[2 * H + u] = dcp * ig * (1 - gg * gg);
          dzv[3 * H + u] = dht * tc * og * (1 - og);
          dc[u] = dcp * fg;
        }
        for (int r = 0; r < 4 * H; ++r) R.dz[(((size_t)l * B + b) * T + t) * 4 * H + r] = dzv[r];
        for (int k = 0; k < H; ++k) {
          double s = 0;
          for (int r = 0; r < 4 * H; ++r) s += (double)whh[l][r * H + k] * dzv[r];
          dh[k] = s;
        }
        if (l > 0)
          for (int k = 0; k < Iin; ++k) {
            double s = 0;
            for (int r = 0; r < 4 * H; ++r) s += (double)wih[l][r * Iin + k] * dzv[r];
            dxn[(size_t)t * H + k] = s;
          }
      }
      dh_in = dxn;
    }
  }
}

static double maxrel(const std::vector<float>& got, const std::vector<double>& ref, size_t n, size_t gst, size_t rst,
                     size_t w) {
  double mx = 0, err = 0;
  for (size_t i = 0; i < n; ++i)
    for (size_t k = 0; k < w; ++k) {
      mx = std::max(mx, std::fabs(ref[i * rst + k]));
      err = std::max(err, std::fabs((double)got[i * gst + k] - ref[i * rst + k]));
    }
  return mx > 0 ? err / mx : err;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1440;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> modes;
  for (int i = 3; i < argc; ++i) modes.push_back(atoi(argv[i]));
  if (modes.empty()) modes = {2, 3, 6, 9};
  const int T = 128, NL = 2;
  const int N = B + 37;  // dataset rows; the batch gathers a random subset
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  const float ws = 1.f / std::sqrt((float)H);
  std::vector<float> x((size_t)N * T * I);
  for (auto& v : x) v = U(rng);
  std::vector<int64_t> lab(N), idx(B);
  for (auto& v : lab) v = rng() % C;
  {
    std::vector<int64_t> perm(N);
    for (int i = 0; i < N; ++i) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    for (int i = 0; i < B; ++i) idx[i] = perm[i];
  }
  std::vector<float> wih[2], whh[2], bih[2], bhh[2], hw(C * H), hb(C);
  for (int l = 0; l < NL; ++l) {
    const int Iin = l == 0 ? I : H;
    wih[l].resize(4 * H * Iin); whh[l].resize(4 * H * H); bih[l].resize(4 * H); bhh[l].resize(4 * H);
    for (auto& v : wih[l]) v = U(rng) * ws;
    for (auto& v : whh[l]) v = U(rng) * ws;
    for (auto& v : bih[l]) v = U(rng) * ws;
    for (auto& v : bhh[l]) v = U(rng) * ws;
  }
  for (auto& v : hw) v = U(rng) * ws;
  for (auto& v : hb) v = U(rng) * ws;

  Ref R;
  reference(NL, B, T, x, idx, lab, wih, whh, bih, bhh, hw, hb, R);
  // the bf16 model's reference: weights, biases and inputs rounded to bf16
  // (the recurrence itself in fp64)
  Ref Rb;
  if (std::find(modes.begin(), modes.end(), 7) != modes.end()) {
    auto rb = [](std::vector<float> v) {
      for (auto& e : v) {
        uint32_t u;
        std::memcpy(&u, &e, 4);
        u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
        std::memcpy(&e, &u, 4);
      }
      return v;
    };
    std::vector<float> wih_b[2], whh_b[2], bih_b[2], bhh_b[2];
    for (int l = 0; l < NL; ++l) { wih_b[l] = rb(wih[l]); whh_b[l] = rb(whh[l]); bih_b[l] = rb(bih[l]); bhh_b[l] = rb(bhh[l]); }
    reference(NL, B, T, rb(x), idx, lab, wih_b, whh_b, bih_b, bhh_b, hw, hb, Rb);
  }

  auto up = [](const void* src, size_t bytes) {
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
    return d;
  };
  float* dx = (float*)up(x.data(), x.size() * 4);
  int64_t* didx = (int64_t*)up(idx.data(), idx.size() * 8);
  int64_t* dlab = (int64_t*)up(lab.data(), lab.size() * 8);
  float *dwih[2], *dwhh[2], *dbih[2], *dbhh[2];
  for (int l = 0; l < NL; ++l) {
    dwih[l] = (float*)up(wih[l].data(), wih[l].size() * 4);
    dwhh[l] = (float*)up(whh[l].data(), whh[l].size() * 4);
    dbih[l] = (float*)up(bih[l].data(), bih[l].size() * 4);
    dbhh[l] = (float*)up(bhh[l].data(), bhh[l].size() * 4);
  }
  float* dhw = (float*)up(hw.data(), hw.size() * 4);
  float* dhb = (float*)up(hb.data(), hb.size() * 4);
  const size_t n_act = (size_t)NL * B * T * 5 * H + PDRNN_DW_PAD_ROWS * 5 * H;
  const size_t n_h = H + (size_t)NL * B * T * H + PDRNN_DW_PAD_ROWS * H;
  const int xg_ld = 12;
  const size_t n_xg = ((size_t)B * T + PDRNN_DW_PAD_ROWS) * xg_ld + 256;
  const int PH = C * H + C + 3;
  float *act, *hbuf, *xg, *hslab, *dhtop, *hn, *cn;
  CK(hipMalloc(&act, n_act * 4)); CK(hipMalloc(&hbuf, n_h * 4)); CK(hipMalloc(&xg, n_xg * 4));
  CK(hipMalloc(&hslab, (size_t)B * PH * 4)); CK(hipMalloc(&dhtop, (size_t)B * H * 4));
  CK(hipMalloc(&hn, (size_t)NL * B * H * 4)); CK(hipMalloc(&cn, (size_t)NL * B * H * 4));
  CK(hipMemset(hbuf, 0, n_h * 4));
  CK(hipMemset(xg, 0, n_xg * 4));
  // dW slab (P = parameter count of the stack)
  int64_t P = 0, off_wih[2], off_whh[2], off_bih[2], off_bhh[2];
  for (int l = 0; l < NL; ++l) {
    const int Iin = l == 0 ? I : H;
    off_wih[l] = P; P += 4 * H * Iin; off_whh[l] = P; P += 4 * H * H;
    off_bih[l] = P; P += 4 * H; off_bhh[l] = P; P += 4 * H;
  }
  const int chunks = pdrnn_lstm_small_dw_chunks(H, NL, B, T);
  float* slab;
  CK(hipMalloc(&slab, (size_t)std::max(std::max(chunks, 1), B) * P * 4));  // (mode 4: one row per sequence)

  PdrnnLstmSmallFwdArgs f{};
  f.x = dx; f.idx = didx; f.x_sb = (int64_t)T * I; f.x_st = I;
  for (int l = 0; l < NL; ++l) { f.w_ih[l] = dwih[l]; f.w_hh[l] = dwhh[l]; f.b_ih[l] = dbih[l]; f.b_hh[l] = dbhh[l]; }
  f.hseq = hbuf + H; f.act = act; f.hn = hn; f.cn = cn;
  f.head_w = dhw; f.head_b = dhb; f.labels = dlab; f.slab = hslab; f.dh_top = dhtop;
  f.slab_P = PH; f.head_off_w = 0; f.head_off_b = C * H; f.stat_off = C * H + C;
  f.inv_batch = 1.f / B; f.C = C; f.B = B; f.T = T; f.I = I; f.NL = NL;
  f.xg_out = xg; f.xg_ld = xg_ld;

  PdrnnLstmSmallBwdArgs bk{};
  bk.x = f.x; bk.idx = f.idx; bk.x_sb = f.x_sb; bk.x_st = f.x_st;
  for (int l = 0; l < NL; ++l) {
    bk.w_ih[l] = dwih[l]; bk.w_hh[l] = dwhh[l];
    bk.off_wih[l] = off_wih[l]; bk.off_whh[l] = off_whh[l]; bk.off_bih[l] = off_bih[l]; bk.off_bhh[l] = off_bhh[l];
  }
  bk.hseq = f.hseq; bk.act = act; bk.dhn = dhtop; bk.dhn_top_only = 1;
  bk.slab = slab; bk.P = P; bk.B = B; bk.T = T; bk.I = I; bk.NL = NL;
  bk.dg_out = act; bk.dg_st = 5 * H; bk.xg_out = xg; bk.xg_ld = xg_ld;

  PdrnnLstmSmallDwArgs dw{};
  dw.xg = xg; dw.xg_ld = xg_ld; dw.hseq = f.hseq; dw.dg = act; dw.dg_st = 5 * H; dw.slab = slab; dw.P = P;
  for (int l = 0; l < NL; ++l) {
    dw.off_wih[l] = off_wih[l]; dw.off_whh[l] = off_whh[l]; dw.off_bih[l] = off_bih[l]; dw.off_bhh[l] = off_bhh[l];
  }
  dw.B = B; dw.T = T; dw.I = I; dw.NL = NL; dw.chunks = chunks;

  // SW_STAMPS=1 (with a -DSW_STAMPS probe build): per-workgroup stamps
  uint64_t* stamps = nullptr;
  const bool want_stamps = getenv("SW_STAMPS") != nullptr;
  if (want_stamps) {
    CK(hipMalloc(&stamps, (size_t)B * 8 * 8 + 4096));  // + the MB_DEBUG dump area
    CK(hipMemset(stamps, 0, (size_t)B * 8 * 8 + 4096));
    f.stamps = stamps;
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));

  std::vector<float> h_act(n_act), h_h(n_h), h_dht((size_t)B * H);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("B=%d T=%d NL=%d CUs=%d reps=%d\n", B, T, NL, cus, reps);
  for (int mode : modes) {
    const bool old = mode == 9;
    const bool mb = false;
    const bool rdw = mode == 4 || mode == 8;  // the backward forms the dW itself (no dz stores, no dW launch)
    const Ref& RR = mb ? Rb : R;
    const double tol = mb ? 3e-2 : 1e-4;
    const int nb_old_f = 1, sp_old_f = B > 1024 ? 2 : 1;
    const int nb_old_b = old ? pdrnn_lstm_small_bwd_dwout_nb(H, NL, T, B) : 1;
    const int grid_old_b = old ? pdrnn_lstm_small_bwd_dwout_grid(H, NL, T, B, nb_old_b) : 0;
    auto run_fwd = [&]() {
      if (old) CK(pdrnn_lstm_small_fwd(&f, H, nb_old_f, sp_old_f, 1, st));
      else CK(pdrnn_lstm_sw_fwd(&f, mode == 4 ? 2 : mode == 8 ? 5 : mode, st));  // 4: backward-only map
    };
    auto run_bwd = [&]() {
      if (old) CK(pdrnn_lstm_small_bwd_dwout(&bk, H, grid_old_b, nb_old_b, st));
      else CK(pdrnn_lstm_sw_bwd(&bk, mode == 6 ? 3 : mode == 8 ? 4 : mode == 5 ? 2 : mode, st));  // 8: fwd 5 + bwd 4
    };
    // correctness: one forward, check; one backward, check
    CK(hipMemsetAsync(act, 0, n_act * 4, st));
    run_fwd();
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h_act.data(), act, n_act * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_h.data(), hbuf, n_h * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_dht.data(), dhtop, (size_t)B * H * 4, hipMemcpyDeviceToHost));
    const size_t rows = (size_t)NL * B * T;
    std::vector<float> hseq_only(h_h.begin() + H, h_h.begin() + H + rows * H);
    const double e_act = maxrel(h_act, RR.act, rows, 5 * H, 5 * H, 5 * H);
    const double e_h = maxrel(hseq_only, RR.hseq, rows, H, H, H);
    const double e_dht = maxrel(h_dht, RR.dhtop, B, H, H, H);
    if (getenv("PROBE_DUMP") && mb && want_stamps) {  // MB_DEBUG build: the h image of step 0, tile 0
      std::vector<uint32_t> d(256), wa(256);
      CK(hipMemcpy(d.data(), reinterpret_cast<uint32_t*>(stamps) + 256, 1024, hipMemcpyDeviceToHost));
      CK(hipMemcpy(wa.data(), reinterpret_cast<uint32_t*>(stamps) + 512, 1024, hipMemcpyDeviceToHost));
      int badw = 0;
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const uint32_t wv = wa[lane * 4 + j / 2];
          const uint32_t bits = (j & 1 ? wv >> 16 : wv & 0xFFFF) << 16;
          float got;
          std::memcpy(&got, &bits, 4);
          const int ai = lane & 15, row = (ai & 3) * H + 8 * (ai >> 2) + 0, k = 8 * (lane >> 4) + j;
          const float ref = whh[0][row * H + k];
          if (std::fabs(got - ref) > 0.01f && badw++ < 6) printf("  W_hh frag lane %d j %d got %.4f ref %.4f\n", lane, j, got, ref);
        }
      printf("  W_hh A fragment (wave 0, m-tile 0): %d of 512 off\n", badw);
      int bad = 0;
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const uint32_t wv = d[lane * 4 + j / 2];
          const uint32_t bits = (j & 1 ? wv >> 16 : wv & 0xFFFF) << 16;
          float got;
          std::memcpy(&got, &bits, 4);
          const int n = lane & 15, u = 8 * (lane >> 4) + j;
          const double ref = RR.hseq[((size_t)n * T + 0) * H + u];
          if (std::fabs(got - ref) > 0.02 && bad++ < 8) printf("  img n=%d u=%d got %.4f ref %.4f\n", n, u, got, ref);
        }
      printf("  h image step 0: %d of 512 off\n", bad);
    }
    if (getenv("PROBE_DUMP") && e_act > tol) {  // first mismatching activations: (l, b, t, slot)
      int shown = 0;
      for (size_t r = 0; r < rows && shown < 12; ++r)
        for (int k = 0; k < 5 * H && shown < 12; ++k) {
          const double ref = RR.act[r * 5 * H + k], got = h_act[r * 5 * H + k];
          if (std::fabs(got - ref) > 0.1) {
            printf("  act l=%zu b=%zu t=%zu slot=%d got %.4f ref %.4f\n", r / ((size_t)B * T), (r / T) % B, r % T, k,
                   got, ref);
            ++shown;
          }
        }
    }
    run_bwd();
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h_act.data(), act, n_act * 4, hipMemcpyDeviceToHost));
    const double e_dz = rdw ? 0.0 : maxrel(h_act, RR.dz, rows, 5 * H, 4 * H, 4 * H);  // (4: no dz stores)
    // the summed weight gradients (slab rows), against the first mode's
    {
      int nrows = B;
      if (!rdw) {
        CK(pdrnn_lstm_small_dw(&dw, H, st));
        nrows = chunks;
      }
      CK(hipStreamSynchronize(st));
      std::vector<float> hs((size_t)nrows * P);
      CK(hipMemcpy(hs.data(), slab, hs.size() * 4, hipMemcpyDeviceToHost));
      std::vector<double> sum(P, 0.0);
      for (int r = 0; r < nrows; ++r)
        for (int64_t k = 0; k < P; ++k) sum[k] += hs[(size_t)r * P + k];
      static std::vector<double> first;
      if (first.empty()) first = sum;
      double mx = 0, err = 0;
      for (int64_t k = 0; k < P; ++k) { mx = std::max(mx, std::fabs(first[k])); err = std::max(err, std::fabs(sum[k] - first[k])); }
      printf("  dW sum vs first mode: max rel %.2e\n", mx > 0 ? err / mx : err);
    }
    // timing
    for (int w = 0; w < 3; ++w) { run_fwd(); run_bwd(); if (!rdw) CK(pdrnn_lstm_small_dw(&dw, H, st)); }
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) run_fwd();
    CK(hipEventRecord(e1, st));
    for (int r = 0; r < reps; ++r) run_bwd();
    CK(hipEventRecord(e2, st));
    for (int r = 0; r < reps; ++r)
      if (!rdw) CK(pdrnn_lstm_small_dw(&dw, H, st));
    CK(hipEventRecord(e3, st));
    CK(hipEventSynchronize(e3));
    float tf = 0, tb = 0, tw = 0;
    CK(hipEventElapsedTime(&tf, e0, e1)); CK(hipEventElapsedTime(&tb, e1, e2)); CK(hipEventElapsedTime(&tw, e2, e3));
    const double uf = 1e3 * tf / reps, ub = 1e3 * tb / reps, uw = 1e3 * tw / reps;
    printf("mode %d%s: fwd %7.1f us (%4.0f cyc/it @2.4)  bwd %7.1f us (%4.0f cyc/it)  dW %6.1f us | err act %.2e h %.2e "
           "dhT %.2e dz %.2e %s\n",
           mode, old ? " (lstm_small)" : mb ? " (bf16 mfma)" : "", uf, uf * 2400.0 / (T + NL - 1), ub,
           ub * 2400.0 / (T + NL - 1), uw, e_act, e_h, e_dht, e_dz,
           (e_act < tol && e_h < tol && e_dht < tol && e_dz < tol) ? "OK" : "MISMATCH");
    if (!rdw && getenv("PROBE_OVERLAP")) {
      // the backward and the dW kernel side by side on two streams (timing
      // only: the dW reads the previous backward's gate gradients)
      static hipStream_t st2 = nullptr;
      static hipEvent_t fk = nullptr, jn = nullptr;
      if (!st2) { CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking)); CK(hipEventCreate(&fk)); CK(hipEventCreate(&jn)); }
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(fk, st));
        CK(hipStreamWaitEvent(st2, fk, 0));
        run_bwd();
        CK(pdrnn_lstm_small_dw(&dw, H, st2));
        CK(hipEventRecord(jn, st2));
        CK(hipStreamWaitEvent(st, jn, 0));
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float to = 0;
      CK(hipEventElapsedTime(&to, e0, e1));
      printf("  overlap: bwd || dW %7.1f us (serial %7.1f)\n", 1e3 * to / reps, ub + uw);
    }
    fflush(stdout);
    if (want_stamps) {
      std::vector<uint64_t> hs((size_t)B * 8);
      CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
      const int g = mode == 3 || mode == 1 ? (B + 1) / 2 : B;
      double lp[2] = {0, 0}, wt[2] = {0, 0}, lo = 0;
      for (int i = 0; i < g; ++i) {
        lo += (double)(hs[i * 8 + 1] - hs[i * 8 + 0]);
        for (int l = 0; l < 2; ++l) { lp[l] += (double)hs[i * 8 + 4 + 2 * l]; wt[l] += (double)hs[i * 8 + 5 + 2 * l]; }
      }
      printf("  stamps (fwd, cycles/step): loop %.0f | layer0 wave %.0f (waits %.0f) | layer1 wave %.0f (waits %.0f)\n",
             lo / g / T, lp[0] / g / T, wt[0] / g / T, lp[1] / g / T, wt[1] / g / T);
      CK(hipMemset(stamps, 0, (size_t)B * 8 * 8));
    }
  }
  return 0;
}
