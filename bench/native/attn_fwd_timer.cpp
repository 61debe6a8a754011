// Stand-alone timer for attention-forward A/B experiments (see attn_bwd_timer.cpp): links ONE
// object defining llmt::launch_attn_fwd and times it on GPT-2 124M's attention shape.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

#ifdef LLMT_ATTN_PROBE
namespace llmt {
void attn_probe_set(unsigned long long* buf);
}
#endif

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  // argv: B [label] [head_dim: 64 or 128; H keeps d_model = 768]
  const int D = argc > 3 ? std::atoi(argv[3]) : 64;
  const int B = argc > 1 ? std::atoi(argv[1]) : 32, T = 1024, H = 768 / D;
  llmt::AttnDims dims;
  dims.B = B;
  dims.T = T;
  dims.H = H;
  dims.hd = D;
  dims.scale = 1.0f / std::sqrt((float)D);
  const size_t nqkv = (size_t)B * T * 3 * H * D, nout = (size_t)B * T * H * D, nrow = (size_t)B * H * T;
  std::vector<unsigned short> h(nqkv);
  unsigned s = 12345;
  for (auto& v : h) {
    s = s * 1664525u + 1013904223u;
    const float f = (((s >> 9) & 0xffff) / 65536.0f - 0.5f) * 4.0f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (unsigned short)(u >> 16);
  }
  void *qkv, *out;
  float* lse;
  CHECK(hipMalloc(&qkv, nqkv * 2));
  CHECK(hipMalloc(&out, nout * 2));
  CHECK(hipMalloc(&lse, nrow * 4));
  CHECK(hipMemcpy(qkv, h.data(), nqkv * 2, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) CHECK(llmt::launch_attn_fwd(qkv, out, lse, dims, llmt::DropoutArgs{}, 0));
  std::vector<float> ms;
  for (int i = 0; i < 30; ++i) {
    CHECK(hipEventRecord(a, 0));
    CHECK(llmt::launch_attn_fwd(qkv, out, lse, dims, llmt::DropoutArgs{}, 0));
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float t;
    CHECK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
#ifdef LLMT_ATTN_PROBE
  {  // per-step cycle anatomy of the (b, h) = 0 workgroups (stamps: csrc/attention_fwd.hip)
    const int nqb = (T + 127) / 128, nev = 64;
    const size_t nwg = (size_t)nqb * B * H;
    const size_t n = (size_t)nqb * 4 * nev + 4 * nwg;
    unsigned long long* dprobe;
    CHECK(hipMalloc(&dprobe, n * 8));
    CHECK(hipMemset(dprobe, 0, n * 8));
    llmt::attn_probe_set(dprobe);
    CHECK(llmt::launch_attn_fwd(qkv, out, lse, dims, llmt::DropoutArgs{}, 0));
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> p(n);
    CHECK(hipMemcpy(p.data(), dprobe, n * 8, hipMemcpyDeviceToHost));
    {  // whole grid: 100 MHz real-time span, shader clock (memtime / realtime), concurrency, WG durations
      const unsigned long long* wg = &p[(size_t)nqb * 4 * nev];
      unsigned long long r0 = ~0ull, r1 = 0;
      double cyc = 0, real = 0;
      std::vector<double> dur(nqb, 0.0);
      for (size_t i = 0; i < nwg; ++i) {
        const unsigned long long* e = &wg[4 * i];
        r0 = std::min(r0, e[2]);
        r1 = std::max(r1, e[3]);
        cyc += (double)(e[1] - e[0]);
        real += (double)(e[3] - e[2]);
        dur[(int)(i % nqb)] += (double)(e[1] - e[0]);
      }
      std::printf("grid span %.1f us (100 MHz realtime) vs %.1f us event-timed; shader clock %.2f GHz; "
                  "%.1f workgroups resident on average\n",
                  (r1 - r0) / 100.0, ms[ms.size() / 2] * 1e3, cyc / real * 0.1,
                  real / (double)(r1 - r0));
      for (int qb = 0; qb < nqb; ++qb) std::printf("  qb=%d mean WG duration %.0f cycles\n", qb, dur[qb] / (B * H));
    }
    for (int qb = 0; qb < nqb; ++qb)
      for (int w = 0; w < 4; ++w) {
        const unsigned long long* e = &p[((size_t)qb * 4 + w) * nev];
        std::printf("probe qb=%d w=%d total=%llu prologue=%llu steps(compute/barrier):", qb, w, e[63] - e[0],
                    e[1] - e[0]);
        unsigned long long prev = e[1];
        for (int it = 0; it < 30 && e[3 + 2 * it] != 0; ++it) {
          const unsigned long long c = e[2 + 2 * it] ? e[2 + 2 * it] - prev : 0;
          std::printf(" %llu/%llu", c, e[3 + 2 * it] - (e[2 + 2 * it] ? e[2 + 2 * it] : prev));
          prev = e[3 + 2 * it];
        }
        std::printf(" tail=%llu\n", e[63] - prev);
      }
  }
#endif
  const double flops = 4.0 * B * H * (double)T * T * D / 2;
  std::printf("{\"kernel\": \"attn_fwd\", \"variant\": \"%s\", \"B\": %d, \"hd\": %d, \"ms\": %.4f, \"TFLOPs\": %.1f}\n",
              argc > 2 ? argv[2] : "?", B, D, ms[ms.size() / 2], flops / ms[ms.size() / 2] / 1e9);
  return 0;
}
