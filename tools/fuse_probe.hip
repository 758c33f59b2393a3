// Multi-role launches (mlkem.hip k_pair / k_seq): which grouping of the batched ML-KEM-768 Encaps /
// Decaps kernels is fastest at 2^20 and 2^16 handshakes.  Every variant is the whole launch
// sequence of one call after the rho copy; hipEvent timing of 10 back-to-back calls, 5 rounds with
// the variants interleaved, after a warm-up that brings the clocks up; the median round is printed.
//   roles alone    xof / front / prf / fix (after its xof) / core / dec / J / G
//   E_sep          xof; front; prf; fix; core                  (every kernel alone)
//   E_pair         xof; front; pair(prf, fix); core            (interleaved multi-role, round-4 head)
//   E_seq          seq(front, xof); seq(fix, prf); core        (latency-bound role's workgroups first)
//   E_seq_prio     the same with the first role at s_setprio 3
//   D_sep          xof; dec; J; G; fix; prf; core
//   D_pair         xof; dec; J; pair(G, fix); prf; core        (round-4 head)
//   D_seq          seq(J, dec, xof); seq(fix, G); prf; core
//   D_seq_b        seq(J, xof); dec; seq(fix, G); prf; core
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fuse_probe.hip -o tools/fuse_probe
#include "../quantum-resistant-p2p_amd/csrc/mlkem.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

namespace qrk {
thread_local KernelTimer* g_timer = nullptr;
thread_local hipError_t g_launch_err = hipSuccess;
}  // namespace qrk
using namespace qrk;
using namespace qrk::mlkem;

constexpr int KK = 3;

template <class R>
struct Prio : R {  // the role's waves at the highest wave priority
  __device__ __forceinline__ void run(unsigned vb, char* lds) const {
    __builtin_amdgcn_s_setprio(3);
    R::run(vb, lds);
  }
};

// role A takes workgroups [0, a.nb), role B the rest
template <class A, class B>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(A::WPE > B::WPE ? A::WPE : B::WPE))) void k_seq(
    A a, B b) {
  constexpr int L = A::LDS > B::LDS ? A::LDS : B::LDS;
  __shared__ __attribute__((aligned(16))) char lds[L > 16 ? L : 16];
  if (blockIdx.x < a.nb)
    a.run(blockIdx.x, lds);
  else
    b.run(blockIdx.x - a.nb, lds);
}
template <class A, class B, class C>
__global__ __launch_bounds__(256) void k_seq3(A a, B b, C c) {
  constexpr int L1 = A::LDS > B::LDS ? A::LDS : B::LDS;
  constexpr int L = L1 > C::LDS ? L1 : C::LDS;
  __shared__ __attribute__((aligned(16))) char lds[L > 16 ? L : 16];
  if (blockIdx.x < a.nb)
    a.run(blockIdx.x, lds);
  else if (blockIdx.x < a.nb + b.nb)
    b.run(blockIdx.x - a.nb, lds);
  else
    c.run(blockIdx.x - a.nb - b.nb, lds);
}

template <class R>
void one(const R& r) {
  if (r.nb) hipLaunchKernelGGL((k_role<R>), dim3(r.nb), dim3(256), 0, 0, r);
}
template <class A, class B>
void pair(const A& a, const B& b) {
  hipLaunchKernelGGL((k_pair<A, B>), dim3(a.nb + b.nb), dim3(256), 0, 0, a, b);
}
template <class A, class B>
void seq(const A& a, const B& b) {
  hipLaunchKernelGGL((k_seq<A, B>), dim3(a.nb + b.nb), dim3(256), 0, 0, a, b);
}
template <class A, class B, class C>
void seq3(const A& a, const B& b, const C& c) {
  hipLaunchKernelGGL((k_seq3<A, B, C>), dim3(a.nb + b.nb + c.nb), dim3(256), 0, 0, a, b, c);
}

__global__ void k_fill(uint64_t* p, size_t n, uint64_t s) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n) p[t] = 0x9E3779B97F4A7C15ull * (t + s) ^ (t << 29);
}
void fill(void* p, size_t bytes, uint64_t s) {
  const size_t w = bytes / 8;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((w + 255) / 256)), dim3(256), 0, 0, (uint64_t*)p, w, s);
}

int main() {
  const size_t NMAX = 1 << 20;
  void* scratch;
  uint8_t *pk, *sk, *coins, *ss, *ct;
  int32_t* status;
  hipMalloc(&scratch, scratch_words(KK, NMAX) * 8);
  hipMalloc(&pk, NMAX * P<KK>::PK);
  hipMalloc(&sk, NMAX * P<KK>::SK);
  hipMalloc(&ct, NMAX * P<KK>::CT);
  hipMalloc(&coins, NMAX * 32);
  hipMalloc(&ss, NMAX * 32);
  hipMalloc(&status, NMAX * 4);
  fill(pk, NMAX * P<KK>::PK, 1);
  fill(sk, NMAX * P<KK>::SK, 5);
  fill(ct, NMAX * P<KK>::CT, 6);
  fill(coins, NMAX * 32, 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"alg\": \"ML-KEM-768\", \"unit\": \"ms per call (median of 5 rounds of 10)\", \"ms\": {");
  for (size_t n : {NMAX, (size_t)1 << 16}) {
    const size_t C = n;
    ScratchView v = carve(scratch, KK, C);
    fill(v.rho, 32 * n, 3);
    fill(v.seeds, 32 * n, 4);
    fill(v.mprime, 32 * n, 7);
    const uint8_t* rho = (const uint8_t*)v.rho;
    const unsigned gblocks = (unsigned)((n + GROUPS - 1) / GROUPS);
    const auto xr = xof_role<KK>(rho, n, C, v);
    const auto fr = fix_role<KK>(rho, n, C, v);
    const RFrontEnc<KK> front{pk, coins, n, ss, v.seeds, blocks_for(n)};
    const RPrf<2, 2> prf{v.seeds, n, C, 2 * KK + 1, KK, v.prf, blocks_for((2 * KK + 1) * C)};
    const RDecrypt<KK> dec{n, ct, sk, v.mprime, gblocks};
    const RJDec<KK> jd{ct, sk, n, v.kbar, blocks_for(n)};
    const RGDec<KK> gd{sk, v.mprime, n, v.seeds, v.kprime, blocks_for(n)};
    const RCore<KK, 0> core0{n, C, v.xof, v.prf, pk, (size_t)P<KK>::PK, coins, 32, ct, status, v.kprime, v.kbar,
                             nullptr, gblocks};
    const RCore<KK, 1> core1{n, C, v.xof, v.prf, sk + 384 * KK, (size_t)P<KK>::SK, (const uint8_t*)v.mprime, 32,
                             ct, nullptr, v.kprime, v.kbar, ss, gblocks};
    const Prio<RFrontEnc<KK>> frontp{front};
    const Prio<RXof<KK, true>> frp{fr};
    auto nf = [&] { hipMemsetAsync(v.nfix, 0, 4, 0); };
    std::vector<std::pair<std::string, std::function<void()>>> vs = {
        {"memset", [&] { nf(); }},
        {"xof", [&] { nf(); one(xr); }},
        {"xof+fix", [&] { nf(); one(xr); one(fr); }},
        {"front", [&] { one(front); }},
        {"prf", [&] { one(prf); }},
        {"core", [&] { one(core0); }},
        {"dec", [&] { one(dec); }},
        {"J", [&] { one(jd); }},
        {"G", [&] { one(gd); }},
        {"core1", [&] { one(core1); }},
        {"E_sep", [&] { nf(); one(xr); one(front); one(prf); one(fr); one(core0); }},
        {"E_pair", [&] { nf(); one(xr); one(front); pair(prf, fr); one(core0); }},
        {"E_seq", [&] { nf(); seq(front, xr); seq(fr, prf); one(core0); }},
        {"E_seq_prio", [&] { nf(); seq(frontp, xr); seq(frp, prf); one(core0); }},
        {"D_sep", [&] { nf(); one(xr); one(dec); one(jd); one(gd); one(fr); one(prf); one(core1); }},
        {"D_pair", [&] { nf(); one(xr); one(dec); one(jd); pair(gd, fr); one(prf); one(core1); }},
        {"D_seq", [&] { nf(); seq3(jd, dec, xr); seq(fr, gd); one(prf); one(core1); }},
        {"D_seq_b", [&] { nf(); seq(jd, xr); one(dec); seq(fr, gd); one(prf); one(core1); }},
    };
    for (int i = 0; i < 10; ++i) vs[11].second();  // warm-up: clocks up
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 5; ++r)
      for (size_t j = 0; j < vs.size(); ++j) {
        vs[j].second();
        hipEventRecord(e0, 0);
        for (int i = 0; i < 10; ++i) vs[j].second();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        t[j].push_back(ms / 10);
      }
    printf("%s\"%zu\": {", n == NMAX ? "" : ", ", n);
    for (size_t j = 0; j < vs.size(); ++j) {
      std::sort(t[j].begin(), t[j].end());
      printf("%s\"%s\": %.4f", j ? ", " : "", vs[j].first.c_str(), t[j][2]);
    }
    printf("}");
  }
  const hipError_t err = hipDeviceSynchronize();
  printf("}, \"hip\": \"%s\"}\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
