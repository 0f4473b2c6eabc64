// Dev probe for the p2m face-skipping path: times p2m_fwd_kernel on the cfg2 workload
// (100k N(0,1) points x 20k N(0,1) faces) with and without Morton order and reports
// how many (wave, face) pairs were skipped.  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -DKL_P2M_PROBE \
//     scripts/dev/p2m_probe.hip -o /tmp/p2m_probe && /tmp/p2m_probe
#include "../../kaolin-windows_amd/csrc/distance.hip"

#include <random>
#include <vector>

namespace kl {
int g_dev_flags = 0;
int g_dev_param[32] = {};
int g_dev_stat[4] = {};
template <typename T>
int acc_finalize(const double *, T *, size_t, bool, hipStream_t, int *) { return 0; }  // backward: unused here
template int acc_finalize<float>(const double *, float *, size_t, bool, hipStream_t, int *);
template int acc_finalize<double>(const double *, double *, size_t, bool, hipStream_t, int *);
void set_error(const std::string &msg) { fprintf(stderr, "error: %s\n", msg.c_str()); }
int fill_async(void *p, int value, size_t bytes, hipStream_t st) { return hipMemsetAsync(p, value, bytes, st) == hipSuccess ? 0 : -2; }
}  // namespace kl

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char **argv) {
  const int64_t P = argc > 1 ? atoll(argv[1]) : 100000, F = argc > 2 ? atoll(argv[2]) : 20000;
  std::mt19937 rng(0);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> hp(P * 3), hf(F * 9);
  for (auto &v : hp) v = nd(rng);
  for (auto &v : hf) v = nd(rng);
  float *dp, *df, *dd;
  int64_t *di;
  int32_t *dt;
  CK(hipMalloc(&dp, P * 12));
  CK(hipMalloc(&df, F * 36));
  CK(hipMalloc(&dd, P * 4));
  CK(hipMalloc(&di, P * 8));
  CK(hipMalloc(&dt, P * 4));
  CK(hipMemcpy(dp, hp.data(), P * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(df, hf.data(), F * 36, hipMemcpyHostToDevice));
  const P2MWs L(P, F, sizeof(float));
  void *ws;
  CK(hipMalloc(&ws, L.bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int targets[] = {6144, 8192, 10240, 12288, 16384, 20480};
  for (int mode = 1; mode < 2 + 5; mode++) {
    unsigned long long z = 0;
    if (mode >= 1) g_p2m_target_blocks = targets[mode - 1];
    for (int rep = 0; rep < 2; rep++) {
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_p2m_skipped), &z, 8));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_p2m_evaluated), &z, 8));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_p2m_pairs), &z, 8));
      CK(hipEventRecord(a, 0));
      int rc = p2m_fwd<float>(P, F, dp, df, dd, di, dt, ws, L.bytes, 0);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      if (rc) return 1;
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      unsigned long long sk, ev, pr;
      CK(hipMemcpyFromSymbol(&sk, HIP_SYMBOL(g_p2m_skipped), 8));
      CK(hipMemcpyFromSymbol(&ev, HIP_SYMBOL(g_p2m_evaluated), 8));
      CK(hipMemcpyFromSymbol(&pr, HIP_SYMBOL(g_p2m_pairs), 8));
      printf("target=%d mode=%s rep=%d  %.3f ms  skipped=%llu evaluated=%llu (%.1f%% skipped) point_pairs=%llu\n",
             g_p2m_target_blocks, mode ? "morton" : "plain", rep, ms, sk, ev, 100.0 * sk / (double)(sk + ev + 1), pr);
    }
  }
  return 0;
}
