// Host CPU cost of one kernel launch call, by kernel shape and launch API (round 6: the single-shot
// KeyGen's host trace puts 3.1 us of CPU in its launch call, an empty-kernel probe 0.6 us).
//   empty: 9 x 320 threads, 2 arguments; big: the same grid, 28 KB of static LDS and the pipelined
//   KeyGen's 10 arguments; each through hipLaunchKernelGGL and through hipModuleLaunchKernel on a
//   hipFunction_t fetched once with hipGetFuncBySymbol.  Per variant: the launch call's CPU time
//   and the round trip to a ticket the kernel stores in fine-grained host memory.  Median / p90 us.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

typedef __attribute__((address_space(1))) unsigned gu32;

__global__ void k_empty(unsigned* resp, unsigned v) {
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store((gu32*)resp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(320) void k_big(size_t n, const uint8_t* a, uint8_t* b, uint8_t* c, void* d, uint32_t* e,
                                             unsigned* resp, unsigned v, uint32_t* f, int g) {
  __shared__ uint32_t lds[7 * 1024];
  for (int i = threadIdx.x; i < 7 * 1024; i += blockDim.x) lds[i] = (uint32_t)i ^ (uint32_t)g;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0 && lds[5] != 0xFFFFFFFFu && n)
    __hip_atomic_store((gu32*)resp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  unsigned *resp, *dresp;
  (void)hipHostMalloc((void**)&resp, 64, hipHostMallocCoherent);
  (void)hipHostGetDevicePointer((void**)&dresp, resp, 0);
  uint8_t* dbuf;
  (void)hipMalloc((void**)&dbuf, 1 << 20);
  hipFunction_t fe = nullptr, fb = nullptr;
  if (hipGetFuncBySymbol(&fe, (const void*)k_empty) != hipSuccess ||
      hipGetFuncBySymbol(&fb, (const void*)k_big) != hipSuccess) {
    printf("{\"error\": \"hipGetFuncBySymbol\"}\n");
    return 1;
  }
  const int N = 2000;
  const char* names[4] = {"empty_ggl", "empty_module", "big_ggl", "big_module"};
  printf("{");
  for (int var = 0; var < 4; ++var) {
    std::vector<double> call, rtt;
    for (int i = 0; i < N + 50; ++i) {
      unsigned v = (unsigned)(var * 1000000 + i + 1);
      size_t n = 1;
      const uint8_t* a = dbuf;
      uint8_t *b = dbuf + 4096, *c = dbuf + 8192;
      void* d = dbuf + 16384;
      uint32_t *e = (uint32_t*)(dbuf + 32768), *f = (uint32_t*)(dbuf + 65536);
      int g = -1;
      const auto t0 = clk::now();
      if (var == 0) {
        hipLaunchKernelGGL(k_empty, dim3(9), dim3(320), 0, st, dresp, v);
      } else if (var == 1) {
        void* args[] = {&dresp, &v};
        (void)hipModuleLaunchKernel(fe, 9, 1, 1, 320, 1, 1, 0, st, args, nullptr);
      } else if (var == 2) {
        hipLaunchKernelGGL(k_big, dim3(9), dim3(320), 0, st, n, a, b, c, d, e, dresp, v, f, g);
      } else {
        void* args[] = {&n, &a, &b, &c, &d, &e, &dresp, &v, &f, &g};
        (void)hipModuleLaunchKernel(fb, 9, 1, 1, 320, 1, 1, 0, st, args, nullptr);
      }
      const auto t1 = clk::now();
      bool ok = true;
      while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != v)
        if (clk::now() - t0 > std::chrono::milliseconds(100)) {
          ok = false;
          break;
        }
      const auto t2 = clk::now();
      (void)hipStreamSynchronize(st);
      if (!ok) {
        printf("\"error\": \"ticket lost in %s\"}\n", names[var]);
        return 1;
      }
      if (i >= 50) {
        call.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        rtt.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
      }
    }
    printf("%s\"%s\": {\"launch_call_us\": {\"p50\": %.2f, \"p90\": %.2f}, \"launch_to_ticket_us\": {\"p50\": %.2f, \"p90\": %.2f}}",
           var ? ", " : "", names[var], pct(call, 0.5), pct(call, 0.9), pct(rtt, 0.5), pct(rtt, 0.9));
  }
  printf(", \"calls\": %d}\n", N);
  return 0;
}
