// 64-bit shift rates on gfx950 and a Keccak-f[1600] whose rotations use them.
//
// Every 64-bit rotation in keccak.cuh is two v_alignbit_b32 (half rate on gfx950,
// profiles/r1/valu_peak_r1b.json).  If v_lshlrev_b64 / v_lshrrev_b64 issue at full rate, a
// rotation becomes one 64-bit shift (the half that needs no merge) + one 32-bit shift + one
// OR: 3 issue slots instead of 4.  This probe measures the shift rates, the permutation rate
// of both variants with the state in registers, and checks the variant bit-exact against
// keccak_f on random states.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/rot64_probe tools/rot64_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../quantum-resistant-p2p_amd/csrc/keccak.cuh"

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int ITERS = 4096;

#define MK64(NAME, INSTR)                                                                     \
  __global__ void k_##NAME(uint32_t* out, uint32_t seed) {                                  \
    uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,   \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed;                            \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(INSTR : "+v"(a0) : "v"(b)); asm volatile(INSTR : "+v"(a1) : "v"(b));      \
      asm volatile(INSTR : "+v"(a2) : "v"(b)); asm volatile(INSTR : "+v"(a3) : "v"(b));      \
      asm volatile(INSTR : "+v"(a4) : "v"(b)); asm volatile(INSTR : "+v"(a5) : "v"(b));      \
      asm volatile(INSTR : "+v"(a6) : "v"(b)); asm volatile(INSTR : "+v"(a7) : "v"(b));      \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }
MK64(lshlrev_b64, "v_lshlrev_b64 %0, 7, %0 ; %1")
MK64(lshrrev_b64, "v_lshrrev_b64 %0, 7, %0 ; %1")
MK64(lshl_add_u64, "v_lshl_add_u64 %0, %0, 3, %1")
MK64(mov_b64, "v_mov_b64 %0, %1 ; %0")
MK64(pk_mov_b32, "v_pk_mov_b32 %0, %0, %1 op_sel:[0,1]")

// ---------------------------------------------------------------- Keccak with 64-bit shifts
struct S64 {
  uint64_t a[25];
};

__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t mk(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

template <int N>
__device__ __forceinline__ uint64_t rot(uint64_t x) {
  if constexpr (N == 0) {
    return x;
  } else if constexpr (N == 32) {
    return mk(hi32(x), lo32(x));
  } else if constexpr (N < 32) {
    uint64_t t;  // t.hi = rot.hi exactly; rot.lo = t.lo | hi >> (32 - N)
    asm("v_lshlrev_b64 %0, %2, %1" : "=v"(t) : "v"(x), "i"(N));
    return mk(lo32(t) | (hi32(x) >> (32 - N)), hi32(t));
  } else {
    uint64_t t;  // t.lo = rot.lo exactly; rot.hi = t.hi | lo << (N - 32)
    asm("v_lshrrev_b64 %0, %2, %1" : "=v"(t) : "v"(x), "i"(64 - N));
    return mk(lo32(t), hi32(t) | (lo32(x) << (N - 32)));
  }
}

__device__ __forceinline__ uint64_t x3(uint64_t a, uint64_t b, uint64_t c) {
  return mk(qrk::xor3(lo32(a), lo32(b), lo32(c)), qrk::xor3(hi32(a), hi32(b), hi32(c)));
}

__device__ __forceinline__ uint32_t chi(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;  // a ^ (~b & c)
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xd2" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ void keccak64(S64& s) {
#pragma unroll 1
  for (int r = 0; r < 24; ++r) {
    uint64_t C[5], R[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = x3(x3(s.a[x], s.a[x + 5], s.a[x + 10]), s.a[x + 15], s.a[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) R[x] = rot<1>(C[x]);
#pragma unroll
    for (int i = 0; i < 25; ++i) s.a[i] = x3(s.a[i], C[(i % 5 + 4) % 5], R[(i % 5 + 1) % 5]);
    B[0] = s.a[0];
    B[10] = rot<1>(s.a[1]);
    B[20] = rot<62>(s.a[2]);
    B[5] = rot<28>(s.a[3]);
    B[15] = rot<27>(s.a[4]);
    B[16] = rot<36>(s.a[5]);
    B[1] = rot<44>(s.a[6]);
    B[11] = rot<6>(s.a[7]);
    B[21] = rot<55>(s.a[8]);
    B[6] = rot<20>(s.a[9]);
    B[7] = rot<3>(s.a[10]);
    B[17] = rot<10>(s.a[11]);
    B[2] = rot<43>(s.a[12]);
    B[12] = rot<25>(s.a[13]);
    B[22] = rot<39>(s.a[14]);
    B[23] = rot<41>(s.a[15]);
    B[8] = rot<45>(s.a[16]);
    B[18] = rot<15>(s.a[17]);
    B[3] = rot<21>(s.a[18]);
    B[13] = rot<8>(s.a[19]);
    B[14] = rot<18>(s.a[20]);
    B[24] = rot<2>(s.a[21]);
    B[9] = rot<61>(s.a[22]);
    B[19] = rot<56>(s.a[23]);
    B[4] = rot<14>(s.a[24]);
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        const uint64_t b0 = B[x + 5 * y], b1 = B[(x + 1) % 5 + 5 * y], b2 = B[(x + 2) % 5 + 5 * y];
        s.a[x + 5 * y] = mk(chi(lo32(b0), lo32(b1), lo32(b2)), chi(hi32(b0), hi32(b1), hi32(b2)));
      }
    s.a[0] ^= mk(qrk::KRC_LO[r], qrk::KRC_HI[r]);
  }
}

__global__ __launch_bounds__(256) void k_keccak_ref(uint64_t* out, int perms) {
  qrk::KState s;
  qrk::kzero(s);
  s.a[0].lo = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < perms; ++p) qrk::keccak_f(s);
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) x ^= qrk::kword(s, i);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int U>
__global__ __launch_bounds__(256) void k_keccak_u(uint64_t* out, int perms) {
  qrk::KState s;
  qrk::kzero(s);
  s.a[0].lo = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < perms; ++p) qrk::keccak_fu<U>(s);
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) x ^= qrk::kword(s, i);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void k_keccak_s64(uint64_t* out, int perms) {
  S64 s;
#pragma unroll
  for (int i = 0; i < 25; ++i) s.a[i] = 0;
  s.a[0] = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < perms; ++p) keccak64(s);
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) x ^= s.a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// bit-exactness: random full states through both permutations
__global__ void k_check(const uint64_t* in, uint64_t* o_ref, uint64_t* o_s64) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  qrk::KState s;
  S64 u;
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    const uint64_t w = in[t * 25 + i];
    s.a[i] = {(uint32_t)w, (uint32_t)(w >> 32)};
    u.a[i] = w;
  }
  qrk::keccak_f(s);
  keccak64(u);
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    o_ref[t * 25 + i] = qrk::kword(s, i);
    o_s64[t * 25 + i] = u.a[i];
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("{\"cus\": %d", cus);
  const int blocks = cus * 8, threads = 256;
  uint32_t* d;
  uint64_t* d64;
  CHECK(hipMalloc(&d, (size_t)blocks * threads * 4));
  CHECK(hipMalloc(&d64, (size_t)cus * 16 * 256 * 8));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  struct K {
    const char* name;
    void (*fn)(uint32_t*, uint32_t);
  } ks[] = {{"lshlrev_b64", k_lshlrev_b64}, {"lshrrev_b64", k_lshrrev_b64}, {"lshl_add_u64", k_lshl_add_u64},
            {"mov_b64", k_mov_b64},         {"pk_mov_b32", k_pk_mov_b32}};
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    printf(", \"%s_Ginstr_lane_per_s\": %.1f", k.name, (double)blocks * threads * ITERS * 8 / (best * 1e-3) / 1e9);
  }
  // correctness on random states
  const int nchk = 4096;
  uint64_t *in, *o1, *o2;
  CHECK(hipMallocManaged(&in, nchk * 25 * 8));
  CHECK(hipMallocManaged(&o1, nchk * 25 * 8));
  CHECK(hipMallocManaged(&o2, nchk * 25 * 8));
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < nchk * 25; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    in[i] = x;
  }
  hipLaunchKernelGGL(k_check, dim3(nchk / 256), dim3(256), 0, 0, in, o1, o2);
  CHECK(hipDeviceSynchronize());
  int bad = 0;
  for (int i = 0; i < nchk * 25; ++i) bad += o1[i] != o2[i];
  printf(", \"s64_mismatch_words\": %d", bad);
  const char* vn[] = {"ref", "s64", "u2", "u3", "u4", "u6"};
  for (int v = 0; v < 6; ++v) {
    for (int wpc : {8, 16}) {
      const int kb = cus * wpc, perms = 64;
      void (*fns[])(uint64_t*, int) = {k_keccak_ref, k_keccak_s64, k_keccak_u<2>, k_keccak_u<3>, k_keccak_u<4>, k_keccak_u<6>};
      auto fn = fns[v];
      hipLaunchKernelGGL(fn, dim3(kb), dim3(256), 0, 0, d64, 2);
      CHECK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(fn, dim3(kb), dim3(256), 0, 0, d64, perms);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
      }
      const double p = (double)kb * 256 * perms;
      printf(", \"keccak_%s_wg%d_perms_per_s\": %.4e, \"keccak_%s_wg%d_Tops_at_4320\": %.3f", vn[v], wpc,
             p / (best * 1e-3), vn[v], wpc, p * 4320 / (best * 1e-3) / 1e12);
    }
  }
  printf("}\n");
  return 0;
}
