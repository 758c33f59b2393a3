// Host-side latency floor of one single-shot call on this box: an empty kernel launch followed by
// (a) hipStreamSynchronize, (b) hipEventSynchronize on an event recorded after it, (c) a host
// spin on a pinned flag the kernel writes (system-scope release).  Median microseconds, JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void k_empty() {}
__global__ void k_flag(volatile unsigned* f, unsigned v) {
  __atomic_store_n((unsigned*)f, v, __ATOMIC_RELEASE);
}

static double med(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  unsigned* flag;
  (void)hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent);
  *flag = 0;
  using clk = std::chrono::steady_clock;
  const int N = 300;
  std::vector<double> a, b, c, d;
  for (int i = 0; i < 20; ++i) {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    (void)hipStreamSynchronize(st);
  }
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    auto t1 = clk::now();
    (void)hipStreamSynchronize(st);
    auto t2 = clk::now();
    a.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
    d.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    (void)hipEventRecord(ev, st);
    (void)hipEventSynchronize(ev);
    b.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  for (int i = 0; i < N; ++i) {
    const unsigned v = (unsigned)i + 1;
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag, v);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
    }
    c.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    (void)hipStreamSynchronize(st);
  }
  // per-call host cost of the API calls a single-shot ABI call makes around its launch
  std::vector<double> er, gdc, gd, sd, lfs;
  for (int i = 0; i < N; ++i) {
    const unsigned v = (unsigned)i + 100000;
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag, v);
    auto t1 = clk::now();
    (void)hipEventRecord(ev, st);
    auto t2 = clk::now();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
    }
    auto t3 = clk::now();
    int cnt = 0, dev = 0;
    (void)hipGetDeviceCount(&cnt);
    auto t4 = clk::now();
    (void)hipGetDevice(&dev);
    auto t5 = clk::now();
    (void)hipSetDevice(dev);
    auto t6 = clk::now();
    (void)hipStreamSynchronize(st);
    er.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
    lfs.push_back(std::chrono::duration<double, std::micro>(t3 - t0).count());
    gdc.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
    gd.push_back(std::chrono::duration<double, std::micro>(t5 - t4).count());
    sd.push_back(std::chrono::duration<double, std::micro>(t6 - t5).count());
  }
  printf("{\"launch_only_us\": %.1f, \"launch_stream_sync_us\": %.1f, \"launch_event_sync_us\": %.1f, "
         "\"launch_flag_spin_us\": %.1f, \"event_record_us\": %.2f, \"launch_record_spin_us\": %.1f, "
         "\"get_device_count_us\": %.2f, \"get_device_us\": %.2f, \"set_device_us\": %.2f}\n",
         med(d), med(a), med(b), med(c), med(er), med(lfs), med(gdc), med(gd), med(sd));
  return 0;
}
