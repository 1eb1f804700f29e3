// Stand-alone timing of pdrnn_slab_reduce_adam (kernels/adam.hip) at the
// fused motion step's slab shapes: recurrent dW rows (one per backward
// workgroup or dW chunk) x 14.0k columns, head rows (one per sequence) x
// ~200 columns, with and without the folded Adam update.
//   reduce_probe [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pdrnn/api.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int64_t PA = 13952, PB = 198 + 3, n_out = PA + 198;
  float *A, *Bs, *g, *tail, *p, *m, *v;
  const int64_t maxA = 1440, maxB = 1440;
  CK(hipMalloc(&A, maxA * PA * 4)); CK(hipMalloc(&Bs, maxB * PB * 4));
  CK(hipMalloc(&g, n_out * 4)); CK(hipMalloc(&tail, 64 * 4));
  CK(hipMalloc(&p, n_out * 4)); CK(hipMalloc(&m, n_out * 4)); CK(hipMalloc(&v, n_out * 4));
  CK(hipMemset(A, 0, maxA * PA * 4)); CK(hipMemset(Bs, 0, maxB * PB * 4));
  CK(hipMemset(p, 0, n_out * 4)); CK(hipMemset(m, 0, n_out * 4)); CK(hipMemset(v, 0, n_out * 4));
  PdrnnAdamArgs ad{};
  ad.param = p; ad.exp_avg = m; ad.exp_avg_sq = v; ad.n = n_out;
  ad.lr = 1e-3f; ad.beta1 = 0.9f; ad.beta2 = 0.999f; ad.eps = 1e-8f;
  ad.bias_correction1 = 0.1f; ad.bias_correction2_sqrt = 0.03f; ad.grad_scale = 1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int64_t rowsAs[] = {180, 256, 360, 512, 720};
  const int64_t rowsBs[] = {0, 180, 720, 1440};
  for (int adam = 0; adam < 2; ++adam)
    for (int64_t ra : rowsAs)
      for (int64_t rb : rowsBs) {
        auto run = [&]() {
          CK(pdrnn_slab_reduce_adam(adam ? &ad : nullptr, A, ra, PA, PA, nullptr, rb ? Bs : nullptr, rb, rb ? PB : 0,
                                    n_out, g, tail, nullptr, 0, 1, 0));
        };
        for (int w = 0; w < 5; ++w) run();
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) run();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("adam %d rowsA %5lld rowsB %5lld: %6.2f us  (%.2f MB)\n", adam, (long long)ra, (long long)rb,
               1e3 * ms / reps, ((double)ra * PA + (double)rb * PB) * 4e-6);
      }
  return 0;
}
