// Where does global_load_lds_dwordx3 put each lane's 12 bytes?  One wave loads word-indexed data
// (word i = i) with 12 bytes per lane from lane-contiguous global addresses into an LDS buffer
// pre-filled with 0xFFFFFFFF; the LDS image is dumped: lane l's first word lands at dword index
// (stride / 4) * l.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* src, uint32_t* dump) {
  __shared__ uint32_t buf[64 * 4 + 64];
  for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) buf[i] = 0xFFFFFFFFu;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 3 * threadIdx.x),
                                   (__attribute__((address_space(3))) void*)&buf[0], 12, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) dump[i] = buf[i];
}
int main() {
  uint32_t h[256 + 64], *s, *d;
  for (int i = 0; i < 256 + 64; ++i) h[i] = i;
  hipMalloc(&s, sizeof(h)); hipMalloc(&d, sizeof(h));
  hipMemcpy(s, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 64>>>(s, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // lane l loaded words 3l, 3l+1, 3l+2: find where word 3l sits
  printf("{\"lane_first_word_dword_index\": [");
  for (int l = 0; l < 8; ++l) {
    int pos = -1;
    for (int i = 0; i < 256 + 64; ++i) if (h[i] == (uint32_t)(3 * l)) { pos = i; break; }
    printf("%s%d", l ? ", " : "", pos);
  }
  printf("], \"lds_dwords_0_15\": [");
  for (int i = 0; i < 16; ++i) printf("%s%d", i ? ", " : "", (int)h[i]);
  printf("]}\n");
  return 0;
}
