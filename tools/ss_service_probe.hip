// Single-shot service probe: what would a resident "service" kernel that polls a
// host-mapped request word save against a kernel launch per single-shot call?
//   (a) launch + flag: an empty 9-workgroup kernel (the k_keygen_pipe grid of ML-KEM-768: 3K
//       workgroups of K + 2 waves) stores a ticket in fine-grained host memory; the host spins on it
//   (b) resident, one poller: one workgroup polls the request word (system-scope relaxed loads over
//       PCIe), echoes the ticket back
//   (c) resident, fan-out: workgroup 0 polls the host word and publishes the request in device memory
//       (sc1 store); the other 8 workgroups poll that (sc1 loads), count in with an agent-scope
//       atomic, and the last one to arrive echoes the ticket: the start / finish fan-out a resident
//       multi-workgroup KeyGen would pay on top of (b)
//   (d) resident, all poll: every one of the 9 workgroups polls the host word itself, counts in with
//       an agent-scope atomic, and the last to arrive echoes the ticket (no device-memory hop at the
//       start)
// Every resident wave exits on a stop word, or by itself after 200 ms without a request (bounded
// spins only: the grid always drains).  Median / p90 microseconds, one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_rel(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned long long IDLE_TICKS = 20000000ull;  // 200 ms of the 100 MHz wall clock

__global__ void k_flag(unsigned* resp, unsigned v) {
  if (blockIdx.x == 0 && threadIdx.x == 0) st_sys_rel(resp, v);
}

// host words: req[0] ticket, req[1] stop; resp[0] echoed ticket.  dev: [0] published ticket,
// [1] arrival count (monotonic: ticket t is complete at 8 t arrivals)
// fanout 0: (b); 1: (c); 2: (d)
__global__ void k_service(const unsigned* req, unsigned* resp, unsigned* dev, int fanout) {
  const bool lane0 = threadIdx.x == 0;
  unsigned last = 0;
  unsigned long long t_idle = wall_clock64();
  for (;;) {
    unsigned t = 0, stop = 0;
    if (blockIdx.x == 0 || fanout == 2) {
      if (lane0) {
        t = ld_sys(&req[0]);
        stop = ld_sys(&req[1]);
      }
    } else if (lane0) {
      t = ld_agent(&dev[0]);
      stop = ld_sys(&req[1]);
    }
    t = __shfl(t, 0);
    stop = __shfl(stop, 0);
    if (stop || wall_clock64() - t_idle > IDLE_TICKS) break;
    if (t == last) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    last = t;
    t_idle = wall_clock64();
    if (!fanout) {
      if (lane0) st_sys_rel(resp, t);
      continue;
    }
    if (fanout == 1 && blockIdx.x == 0) {
      if (lane0) st_agent(&dev[0], t);
      continue;
    }
    const unsigned parts = fanout == 2 ? 9u : 8u;
    if (lane0) {
      const unsigned prev = __hip_atomic_fetch_add(&dev[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev + 1 == parts * t) st_sys_rel(resp, t);
    }
  }
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t st, svc;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&svc, hipStreamNonBlocking);
  unsigned *req, *resp, *dev;
  (void)hipHostMalloc((void**)&req, 64, hipHostMallocCoherent);
  (void)hipHostMalloc((void**)&resp, 64, hipHostMallocCoherent);
  (void)hipMalloc((void**)&dev, 64);
  unsigned *dreq, *dresp;
  (void)hipHostGetDevicePointer((void**)&dreq, req, 0);
  (void)hipHostGetDevicePointer((void**)&dresp, resp, 0);
  const int N = 2000;
  std::vector<double> a, b, c, d;
  auto spin = [&](unsigned v) {
    const auto t0 = clk::now();
    while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != v)
      if (clk::now() - t0 > std::chrono::milliseconds(100)) return false;
    return true;
  };
  // (a) launch + flag
  for (int i = 0; i < N + 20; ++i) {
    const unsigned v = 1000000u + (unsigned)i;
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_flag, dim3(9), dim3(320), 0, st, dresp, v);
    const bool ok = spin(v);
    const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    (void)hipStreamSynchronize(st);
    if (!ok) {
      printf("{\"error\": \"launch flag lost\"}\n");
      return 1;
    }
    if (i >= 20) a.push_back(us);
  }
  // (b), (c) resident
  for (int fan = 0; fan < 3; ++fan) {
    req[0] = 0, req[1] = 0, resp[0] = 0;
    (void)hipMemset(dev, 0, 64);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_service, dim3(fan ? 9 : 1), dim3(64), 0, svc, dreq, dresp, dev, fan);
    std::vector<double>& out = fan == 0 ? b : fan == 1 ? c : d;
    bool ok = true;
    for (int i = 1; i <= N + 20 && ok; ++i) {
      const auto t0 = clk::now();
      __atomic_store_n(&req[0], (unsigned)i, __ATOMIC_RELEASE);
      ok = spin((unsigned)i);
      const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      if (i > 20) out.push_back(us);
    }
    __atomic_store_n(&req[1], 1u, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(svc);
    if (!ok) {
      printf("{\"error\": \"resident service lost a request\", \"fanout\": %d}\n", fan);
      return 1;
    }
  }
  printf("{\"launch_flag_us\": {\"p50\": %.2f, \"p90\": %.2f}, \"resident_one_poller_us\": {\"p50\": %.2f, \"p90\": %.2f}, "
         "\"resident_fanout9_us\": {\"p50\": %.2f, \"p90\": %.2f}, \"resident_allpoll9_us\": {\"p50\": %.2f, \"p90\": %.2f}, "
         "\"calls\": %d}\n",
         pct(a, 0.5), pct(a, 0.9), pct(b, 0.5), pct(b, 0.9), pct(c, 0.5), pct(c, 0.9), pct(d, 0.5), pct(d, 0.9), N);
  return 0;
}
