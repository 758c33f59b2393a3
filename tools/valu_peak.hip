// VALU instruction-throughput microbenchmark for gfx950 (MI355X).
//
// Measures, for the instructions the Keccak and NTT kernels are made of, how
// many lane-ops per second the whole chip sustains (8 independent register
// chains per lane, enough waves per SIMD), and Keccak-f[1600] permutations per
// second with the state held in registers (no memory traffic).  The result is
// the measured denominator for bench.py's VALU roofline.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_peak tools/valu_peak.hip
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

#define CHAIN8(OP) \
  OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

__global__ void k_bitop3(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234, c = seed ^ 0x9876;
  for (int i = 0; i < ITERS; ++i) {
#define OPB(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
    CHAIN8(OPB)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234;
  for (int i = 0; i < ITERS; ++i) {
#define OPA(x) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
    CHAIN8(OPA)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_xor(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234;
  for (int i = 0; i < ITERS; ++i) {
#define OPX(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
    CHAIN8(OPX)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mad24(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15, b = seed & 0xFFFF;
  for (int i = 0; i < ITERS; ++i) {
#define OPM(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(b));
    CHAIN8(OPM)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15, b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
#define OPL(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
    CHAIN8(OPL)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}


#define MKK(NAME, INSTR, INIT_B)                                                               \
  __global__ void k_##NAME(uint32_t* out, uint32_t seed) {                                  \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,   \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = INIT_B;                          \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(INSTR : "+v"(a0) : "v"(b)); asm volatile(INSTR : "+v"(a1) : "v"(b));      \
      asm volatile(INSTR : "+v"(a2) : "v"(b)); asm volatile(INSTR : "+v"(a3) : "v"(b));      \
      asm volatile(INSTR : "+v"(a4) : "v"(b)); asm volatile(INSTR : "+v"(a5) : "v"(b));      \
      asm volatile(INSTR : "+v"(a6) : "v"(b)); asm volatile(INSTR : "+v"(a7) : "v"(b));      \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;    \
  }
MKK(mul_lo_u16, "v_mul_lo_u16 %0, %0, %1", seed | 1)
MKK(mul_i32_i24, "v_mul_i32_i24 %0, %0, %1", seed & 0xFFF)
MKK(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1", seed & 0xFFF)
MKK(mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1", seed & 0xFFF)
MKK(mul_f32, "v_mul_f32 %0, %0, %1", 0x3f800001u)
MKK(fma_f32, "v_fma_f32 %0, %0, %1, %1", 0x3f000000u)
MKK(rndne_f32, "v_rndne_f32 %0, %0 ; %1", 0u)
MKK(dot2c_i32_i16, "v_dot2c_i32_i16 %0, %1, %1", seed)
MKK(bcnt, "v_bcnt_u32_b32 %0, %0, %1", seed)
MKK(perm, "v_perm_b32 %0, %0, %1, %1", seed)
MKK(bfe_u32, "v_bfe_u32 %0, %0, 3, 12 ; %1", seed)
MKK(add_u32, "v_add_u32 %0, %0, %1", seed)
MKK(lshl_add, "v_lshl_add_u32 %0, %0, 3, %1", seed)
MKK(ashr, "v_ashrrev_i32 %0, 16, %0 ; %1", seed)
MKK(pk_add_u16, "v_pk_add_u16 %0, %0, %1", seed)
MKK(pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %0, %1", seed)
MKK(fmac_f32, "v_fmac_f32 %0, %1, %1", 0x3f000000u)
MKK(fmaak_f32, "v_fmaak_f32 %0, %0, %1, 0x3f000000", 0x3f000000u)
MKK(add_f32, "v_add_f32 %0, %0, %1", 0x3f000000u)
MKK(cvt_f32_i32, "v_cvt_f32_i32 %0, %0 ; %1", 0u)
MKK(cvt_i32_f32, "v_cvt_i32_f32 %0, %0 ; %1", 0u)
MKK(mad_i32_i16, "v_mad_i32_i16 %0, %0, %1, %1", seed)
MKK(mad_u32_u16, "v_mad_u32_u16 %0, %0, %1, %1", seed)
MKK(mul_hi_i32, "v_mul_hi_i32 %0, %0, %1", seed)
MKK(pk_mad_i16, "v_pk_mad_i16 %0, %0, %1, %1", seed)
MKK(sub_sdwa, "v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0", seed)
MKK(bfe_i32, "v_bfe_i32 %0, %0, 0, 16 ; %1", seed)
MKK(med3_i32, "v_med3_i32 %0, %0, %1, %1", seed)
MKK(cndmask, "v_cndmask_b32 %0, %0, %1, vcc", seed)
MKK(cndmask_e64, "v_cndmask_b32_e64 %0, %0, %1, s[4:5]", seed)
MKK(cmp_cndmask, "v_cmp_gt_u32 vcc, %1, %0\n v_cndmask_b32 %0, %0, %1, vcc", seed)
MKK(cmp_addc, "v_cmp_gt_u32 vcc, %1, %0\n v_addc_co_u32 %0, vcc, 0, %0, vcc", seed)
MKK(sub_ashr, "v_sub_u32 %0, %0, %1\n v_ashrrev_i32 %0, 1, %0", seed)
MKK(and_or, "v_and_or_b32 %0, %0, %1, %1", seed)
MKK(lshl_or, "v_lshl_or_b32 %0, %0, 3, %1", seed)

// 64-bit register (packed fp32) ops: instruction rate (each instruction = 2 fp32 lanes)
#define MKK64(NAME, INSTR, INIT_B)                                                            \
  __global__ void k_##NAME(uint32_t* out, uint32_t seed) {                                  \
    uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,   \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = INIT_B;                          \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(INSTR : "+v"(a0) : "v"(b)); asm volatile(INSTR : "+v"(a1) : "v"(b));      \
      asm volatile(INSTR : "+v"(a2) : "v"(b)); asm volatile(INSTR : "+v"(a3) : "v"(b));      \
      asm volatile(INSTR : "+v"(a4) : "v"(b)); asm volatile(INSTR : "+v"(a5) : "v"(b));      \
      asm volatile(INSTR : "+v"(a6) : "v"(b)); asm volatile(INSTR : "+v"(a7) : "v"(b));      \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }
MKK64(pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %1", 0x3f0000003f000000ull)
MKK64(pk_mul_f32, "v_pk_mul_f32 %0, %0, %1", 0x3f8000003f800000ull)
MKK64(pk_add_f32, "v_pk_add_f32 %0, %0, %1", 0x3f0000003f000000ull)

// Keccak-f[1600] on register state, PERMS permutations per lane
__global__ __launch_bounds__(256) void k_keccak(uint64_t* out, int perms) {
  qrk::KState s;
  qrk::kzero(s);
  s.a[0].lo = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < perms; ++p) qrk::keccak_f(s);
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) x ^= qrk::kword(s, i);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d", prop.name, cus, prop.clockRate);
  const int blocks = cus * 8, threads = 256;  // 8 waves / SIMD resident
  uint32_t* d;
  uint64_t* d64;
  CHECK(hipMalloc(&d, (size_t)blocks * threads * 4));
  CHECK(hipMalloc(&d64, (size_t)blocks * threads * 8 * 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  struct K {
    const char* name;
    void (*fn)(uint32_t*, uint32_t);
  } ks[] = {{"bitop3", k_bitop3}, {"alignbit", k_alignbit}, {"xor", k_xor}, {"mad_u32_u24", k_mad24},
            {"mul_lo_u32", k_mullo}, {"mul_lo_u16", k_mul_lo_u16}, {"mul_i32_i24", k_mul_i32_i24},
            {"mul_u32_u24", k_mul_u32_u24}, {"mul_hi_u32_u24", k_mul_hi_u32_u24}, {"mul_f32", k_mul_f32},
            {"fma_f32", k_fma_f32}, {"rndne_f32", k_rndne_f32}, {"dot2c_i32_i16", k_dot2c_i32_i16}, {"bcnt", k_bcnt},
            {"perm", k_perm}, {"bfe_u32", k_bfe_u32}, {"add_u32", k_add_u32}, {"lshl_add", k_lshl_add}, {"ashr", k_ashr},
            {"pk_add_u16", k_pk_add_u16}, {"pk_mul_lo_u16", k_pk_mul_lo_u16}, {"fmac_f32", k_fmac_f32},
            {"fmaak_f32", k_fmaak_f32}, {"add_f32", k_add_f32}, {"cvt_f32_i32", k_cvt_f32_i32},
            {"cvt_i32_f32", k_cvt_i32_f32}, {"mad_i32_i16", k_mad_i32_i16}, {"mad_u32_u16", k_mad_u32_u16},
            {"mul_hi_i32", k_mul_hi_i32}, {"pk_mad_i16", k_pk_mad_i16}, {"sub_sdwa", k_sub_sdwa},
            {"bfe_i32", k_bfe_i32}, {"med3_i32", k_med3_i32}, {"cndmask", k_cndmask},
            {"cndmask_e64", k_cndmask_e64}, {"cmp_cndmask_pair", k_cmp_cndmask}, {"cmp_addc_pair", k_cmp_addc},
            {"sub_ashr_pair", k_sub_ashr}, {"and_or", k_and_or}, {"lshl_or", k_lshl_or},
            {"pk_fma_f32_instr", k_pk_fma_f32}, {"pk_mul_f32_instr", k_pk_mul_f32}, {"pk_add_f32_instr", k_pk_add_f32}};
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
    const double ops = (double)blocks * threads * ITERS * 8;
    printf(", \"%s_Tops\": %.3f", k.name, ops / (best * 1e-3) / 1e12);
  }
  // Keccak: 4 WGs of 256 per CU x 4 rounds
  for (int wpc : {4, 8, 16}) {
    const int kb = cus * wpc;
    const int perms = 64;
    hipLaunchKernelGGL(k_keccak, dim3(kb), dim3(256), 0, 0, d64, 2);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_keccak, dim3(kb), dim3(256), 0, 0, d64, perms);
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    const double p = (double)kb * 256 * perms;
    printf(", \"keccak_wg%d_perms_per_s\": %.4e, \"keccak_wg%d_Tops_at_4320\": %.3f", wpc, p / (best * 1e-3), wpc,
           p * 4320 / (best * 1e-3) / 1e12);
  }
  printf("}\n");
  return 0;
}
