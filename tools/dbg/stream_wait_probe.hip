// Does hipStreamWaitEvent(A, ev recorded on a non-blocking stream B) order A's next kernel after
// B's work?  B: a ~2 ms busy kernel that then writes flag = token; record ev on B; A waits ev; A: a
// kernel that copies flag to out.  out != token means the wait did not hold.  A = the NULL stream,
// a blocking stream, a non-blocking stream; repeated with fresh and reused events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void busy_then_flag(uint32_t* flag, uint32_t token, uint64_t cycles, uint32_t* sink) {
  uint64_t t0 = clock64();
  uint32_t x = threadIdx.x;
  while (clock64() - t0 < cycles) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) sink[0] = x;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __threadfence();
    *(volatile uint32_t*)flag = token;
  }
}
__global__ void read_flag(const uint32_t* flag, uint32_t* out, int i) {
  if (threadIdx.x == 0) out[i] = *(volatile const uint32_t*)flag;
}

int main() {
  uint32_t *flag, *out, *sink;
  hipMalloc(&flag, 4); hipMalloc(&out, 4096); hipMalloc(&sink, 4);
  hipMemset(flag, 0, 4); hipMemset(out, 0, 4096);
  hipStream_t B, Ablk, Anb;
  hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&Ablk, hipStreamDefault);
  hipStreamCreateWithFlags(&Anb, hipStreamNonBlocking);
  hipEvent_t reuse;
  hipEventCreateWithFlags(&reuse, hipEventDisableTiming);
  const char* names[3] = {"null", "blocking", "nonblocking"};
  hipStream_t As[3] = {0, Ablk, Anb};
  int bad[3][2] = {};
  const int R = 40;
  for (int mode = 0; mode < 3; ++mode) {
    for (int fresh = 0; fresh < 2; ++fresh) {
      for (int r = 0; r < R; ++r) {
        const uint32_t token = 1000 * (mode * 2 + fresh) + r + 1;
        hipEvent_t ev = reuse;
        if (fresh) hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        busy_then_flag<<<256, 256, 0, B>>>(flag, token, 2000000ull, sink);  // ~1 ms at 2 GHz
        hipEventRecord(ev, B);
        hipStreamWaitEvent(As[mode], ev, 0);
        read_flag<<<1, 64, 0, As[mode]>>>(flag, out, r);
        if (fresh) hipEventDestroy(ev);
        hipDeviceSynchronize();
        uint32_t h = 0;
        hipMemcpy(&h, out + r, 4, hipMemcpyDeviceToHost);
        if (h != token) ++bad[mode][fresh];
      }
    }
  }
  // pipelined: every (B work, record, A wait, A read) enqueued back to back, one sync at the end;
  // tokens increase, so a read that did not wait shows a token below its own
  int pbad[3] = {};
  for (int mode = 0; mode < 3; ++mode) {
    hipMemset(out, 0, 4096);
    hipEvent_t evs[R];
    for (int r = 0; r < R; ++r) {
      hipEventCreateWithFlags(&evs[r], hipEventDisableTiming);
      busy_then_flag<<<256, 256, 0, B>>>(flag, 100000 * (mode + 1) + r + 1, 2000000ull, sink);
      hipEventRecord(evs[r], B);
      hipStreamWaitEvent(As[mode], evs[r], 0);
      read_flag<<<1, 64, 0, As[mode]>>>(flag, out, r);
    }
    hipDeviceSynchronize();
    uint32_t h[R];
    hipMemcpy(h, out, 4 * R, hipMemcpyDeviceToHost);
    for (int r = 0; r < R; ++r) {
      if (h[r] < 100000u * (mode + 1) + r + 1) ++pbad[mode];
      hipEventDestroy(evs[r]);
    }
  }
  for (int mode = 0; mode < 3; ++mode)
    printf("{\"A\": \"%s\", \"pipelined_misses\": %d, \"trials\": %d}\n", names[mode], pbad[mode], R);
  // reverse direction: the producer is the NULL stream (the caller's stream under PyTorch), the
  // waiter a non-blocking library stream (the launchers' forks), pipelined
  {
    int rbad = 0;
    hipMemset(out, 0, 4096);
    hipDeviceSynchronize();
    hipEvent_t evs[R];
    for (int r = 0; r < R; ++r) {
      hipEventCreateWithFlags(&evs[r], hipEventDisableTiming);
      busy_then_flag<<<256, 256, 0, 0>>>(flag, 900000 + r + 1, 2000000ull, sink);
      hipEventRecord(evs[r], 0);
      hipStreamWaitEvent(Anb, evs[r], 0);
      read_flag<<<1, 64, 0, Anb>>>(flag, out, r);
    }
    hipDeviceSynchronize();
    uint32_t h[R];
    hipMemcpy(h, out, 4 * R, hipMemcpyDeviceToHost);
    for (int r = 0; r < R; ++r) {
      if (h[r] < 900000u + r + 1) ++rbad;
      hipEventDestroy(evs[r]);
    }
    printf("{\"producer\": \"null\", \"waiter\": \"nonblocking\", \"pipelined_misses\": %d, \"trials\": %d}\n", rbad, R);
  }
  for (int mode = 0; mode < 3; ++mode)
    printf("{\"A\": \"%s\", \"reused_event_misses\": %d, \"fresh_event_misses\": %d, \"trials\": %d}\n", names[mode],
           bad[mode][0], bad[mode][1], R);
  return 0;
}
