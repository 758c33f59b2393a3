// Multi-role launches (mlkem.hip k_pair / k_seq): which grouping of the batched ML-KEM-768 Encaps /
// Decaps kernels is fastest at 2^20, 2^18, 2^16 and 2^14 handshakes.  Every variant is the whole launch
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
//   E_m1 / E_m2    seq(front, xof); pair(prf, fix) / xof; front; seq(fix, prf)  (+ core)
//   D_c            seq(J, xof); seq(fix, dec); G; prf; core
//   D_d            seq(J, dec, xof); G; seq(fix, prf); core
//   D_e            seq(J, dec, xof); pair(G, fix); prf; core
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

// the round-4 head's interleaved multi-role kernel: role B takes workgroup w iff
// floor((w + 1) nb_B / N) > floor(w nb_B / N), N = nb_A + nb_B
template <class A, class B>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(A::WPE > B::WPE ? A::WPE : B::WPE))) void k_pair(
    A a, B b) {
  constexpr int L = A::LDS > B::LDS ? A::LDS : B::LDS;
  __shared__ __attribute__((aligned(16))) char lds[L > 16 ? L : 16];
  const uint64_t N = (uint64_t)a.nb + b.nb, w = blockIdx.x;
  const uint32_t tb = (uint32_t)(w * b.nb / N), tb1 = (uint32_t)((w + 1) * b.nb / N);
  if (tb1 != tb)
    b.run(tb, lds);
  else
    a.run((uint32_t)w - tb, lds);
}
// role A takes workgroups [0, a.nb), role B the rest (as mlkem.hip k_multi)
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

int main(int argc, char** argv) {
  // optional: one log2 batch size and the number of rounds (default: the four sizes, 5 rounds)
  const int lb = argc > 1 ? atoi(argv[1]) : 0, rounds = argc > 2 ? atoi(argv[2]) : 5;
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
  printf("{\"alg\": \"ML-KEM-768\", \"unit\": \"ms per call (median of the rounds of 10 calls)\", \"ms\": {");
  std::vector<size_t> sizes = {NMAX, (size_t)1 << 18, (size_t)1 << 16, (size_t)1 << 14};
  if (lb) sizes = {(size_t)1 << lb};
  bool first = true;
  for (size_t n : sizes) {
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
        {"xof_occ4", [&] { nf(); hipLaunchKernelGGL((k_role<RXof<KK, false>>), dim3(xr.nb), dim3(256), 40 * 1024 - XOF_LDS, 0, xr); }},
        {"xof_occ3", [&] { nf(); hipLaunchKernelGGL((k_role<RXof<KK, false>>), dim3(xr.nb), dim3(256), 53 * 1024 - XOF_LDS, 0, xr); }},
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
        {"E_m1", [&] { nf(); seq(front, xr); pair(prf, fr); one(core0); }},
        {"E_m2", [&] { nf(); one(xr); one(front); seq(fr, prf); one(core0); }},
        {"D_sep", [&] { nf(); one(xr); one(dec); one(jd); one(gd); one(fr); one(prf); one(core1); }},
        {"D_pair", [&] { nf(); one(xr); one(dec); one(jd); pair(gd, fr); one(prf); one(core1); }},
        {"D_seq", [&] { nf(); seq3(jd, dec, xr); seq(fr, gd); one(prf); one(core1); }},
        {"D_seq_b", [&] { nf(); seq(jd, xr); one(dec); seq(fr, gd); one(prf); one(core1); }},
        {"D_c", [&] { nf(); seq(jd, xr); seq(fr, dec); one(gd); one(prf); one(core1); }},
        {"D_d", [&] { nf(); seq3(jd, dec, xr); one(gd); seq(fr, prf); one(core1); }},
        {"D_e", [&] { nf(); seq3(jd, dec, xr); pair(gd, fr); one(prf); one(core1); }},
    };
    for (int i = 0; i < 10; ++i) vs[13].second();  // warm-up: clocks up
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
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
    printf("%s\"%zu\": {", first ? "" : ", ", n);
    first = false;
    for (size_t j = 0; j < vs.size(); ++j) {
      std::sort(t[j].begin(), t[j].end());
      printf("%s\"%s\": %.4f", j ? ", " : "", vs[j].first.c_str(), t[j][rounds / 2]);
    }
    printf("}");
  }
  const hipError_t err = hipDeviceSynchronize();
  printf("}, \"hip\": \"%s\"}\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
