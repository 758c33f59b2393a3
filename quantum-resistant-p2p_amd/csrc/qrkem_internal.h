// Internal host-side interface between the C-ABI (abi.cpp) and the kernel
// launchers (mlkem.hip, frodo.hip, util.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace qrk {

enum class Family { MLKEM, FRODO, HQC };

struct AlgInfo {
  const char* name;
  Family family;
  int level;        // claimed NIST level (OQS_KEM.claimed_nist_level)
  int k;            // ML-KEM module rank, Frodo n, or HQC security bits (128/192/256)
  size_t pk, sk, ct, ss;
  size_t kp_coins, enc_coins;  // bytes drawn by one keypair / encaps randombytes call
  bool aes;         // Frodo A generated with AES-128 (else SHAKE128)
  bool enabled;     // has a HIP implementation in this build
};

const AlgInfo* find_alg(const char* name);
int alg_count();
const AlgInfo* alg_at(int i);

// Optional per-kernel HIP-event timing (qrk_ctx_profile): when a context has
// profiling enabled, every QRK_LAUNCH brackets the launch with two events on the
// launch stream; durations are summed per kernel name.
struct KernelTimer {
  virtual void before(const char* name, hipStream_t st) = 0;
  virtual void after(const char* name, hipStream_t st) = 0;
  virtual ~KernelTimer() = default;
};
extern thread_local KernelTimer* g_timer;
// First kernel-launch error of the current library call (HIP resets its last-error state on every
// later successful API call, so a failed launch followed by successful ones would otherwise go
// unnoticed); run_batch clears it before each chunk and fails the call when it is set.
extern thread_local hipError_t g_launch_err;

// stream / event / memset calls inside the launchers: a failure joins g_launch_err
inline void qrk_chk(hipError_t e) {
  if (e != hipSuccess && g_launch_err == hipSuccess) g_launch_err = e;
}

#define QRK_LAUNCH(NAME, ST, ...)                   \
  do {                                              \
    if (::qrk::g_timer) ::qrk::g_timer->before(NAME, ST); \
    hipLaunchKernelGGL(__VA_ARGS__);                \
    {                                               \
      const hipError_t qrk_le_ = hipGetLastError(); \
      if (qrk_le_ != hipSuccess && qrk_le_ != hipErrorNotReady && ::qrk::g_launch_err == hipSuccess) \
        ::qrk::g_launch_err = qrk_le_;                \
    }                                               \
    if (::qrk::g_timer) ::qrk::g_timer->after(NAME, ST);  \
  } while (0)

// Device scratch owned by a context.  Grown on demand, never shrunk.
struct Scratch {
  void* base = nullptr;
  size_t bytes = 0;
};

// Per-chunk scratch requirement (bytes) for `chunk` handshakes of `a`.
size_t mlkem_scratch_bytes(const AlgInfo& a, size_t chunk);
size_t frodo_scratch_bytes(const AlgInfo& a, size_t chunk);
size_t hqc_scratch_bytes(const AlgInfo& a, size_t chunk);
// Zero the per-handshake key-material records one chunk of n handshakes left in scratch
// (ML-KEM: seeds, m', K', Kbar; FrodoKEM: seedSE || k || pkh || mu', the hashed key; HQC: the
// K-hash message m || u || v and m'), stream-ordered: called after every chunk.
hipError_t mlkem_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st);
// byte offset and length of the ML-KEM per-handshake records (seeds | m' | K' | Kbar) in the
// scratch of a chunk of C handshakes (tests: qrk_dbg_mlkem_records_residue)
void mlkem_records_span(const AlgInfo& a, size_t C, size_t* off, size_t* bytes);
// ML-KEM batches up to this size run as one launch per operation with no scratch key material
size_t mlkem_small_max();
// ML-KEM KeyGen batches up to this size run one workgroup per SampleNTT / PRF item (latency)
size_t mlkem_kg_multi_max();
// flag / counter words of the single-shot multi-workgroup KeyGen (ctx->kg_cnt)
size_t mlkem_kg_flag_words();
// bytes of the batched sampled matrix of a chunk of `chunk` handshakes (Streams::xof_keep)
size_t mlkem_matrix_bytes(const AlgInfo& a, size_t chunk);
// bytes at the start of the scratch that the n <= mlkem_kg_multi_max() KeyGen kernels use
size_t mlkem_kg_scratch_bytes();
// tests only (qrk_dbg_kg_late): the k_keygen_pipe workgroup role (PRF item or t_hat row) that
// publishes past every bounded wait, -1 (default) none
extern int g_kg_dbg_late;
// tests only (qrk_dbg_fail_after_flip): batched ML-KEM Encaps / Decaps chunks <= 2^15 fail right after
// the fix-up counter parity flip, before any launch (0 = off)
extern int g_dbg_fail_after_flip;
hipError_t frodo_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st);
hipError_t hqc_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st);

// Launch context of one call: every kernel of the call runs on `main`, the caller's stream (no
// side streams, no cross-stream events: a call is stream-ordered and never blocks the host).
struct Streams {
  hipStream_t main = nullptr;
  // serial schedule: one kernel per launch (per-kernel timings in isolation); otherwise
  // independent kernels of one operation share multi-role launches (ML-KEM, mlkem.hip)
  bool serial = false;
  // single-shot completion flag (fine-grained host memory, device address): the one-launch ML-KEM
  // kernels store `ticket` there once their outputs are visible to the host
  uint32_t* done = nullptr;
  uint32_t ticket = 0;
  // per-handshake arrival counters of the multi-workgroup single-shot ML-KEM KeyGen (device,
  // QRK_KG_MULTI_MAX words, zero between calls: the last workgroup of a handshake resets its word)
  uint32_t* kg_cnt = nullptr;
  // host-pointer ML-KEM KeyGen of n <= mlkem_kg_multi_max(): the call's error word (fine-grained host
  // memory, device address, zeroed by the host before the launch).  When set, k_keygen_pipe runs and
  // stores 1 there if a bounded cross-workgroup wait expired; the host then fails the call.
  uint32_t* kg_err = nullptr;
  // single-shot ML-KEM (n == 1, host-pointer call): the public input in host memory (Encaps: pk;
  // Decaps: c), passed as a kernel argument instead of read over PCIe.  Secret inputs are never
  // passed by value: the runtime's kernel-argument pool is not wiped.
  const uint8_t* host_in1 = nullptr;
  // batched ML-KEM Encaps / Decaps at chunks <= 2^15: the context's two SampleNTT fix-up counters
  // (device, zero at allocation) and which one the next call counts into (host; the call flips it
  // and its first launch zeroes the other word, mlkem.hip rho_source).  Set only by run_batch, which
  // re-zeroes both words after any failed chunk (qrk_ctx::fixc_dirty).
  uint32_t* fixc = nullptr;
  int* fixp = nullptr;
  // batched ML-KEM (one chunk, n > mlkem_small_max()), the handshake driver's expanded-key reuse:
  // KeyGen writes its sampled matrix A_hat (SampleNTT(rho || x || y), the batched tiled layout,
  // mlkem_matrix_bytes) to xof_keep instead of the scratch; Decaps of the same keys, same chunk size,
  // takes it from xof_given and skips its own SampleNTT (A_hat is a function of rho alone).
  uint64_t* xof_keep = nullptr;
  const uint64_t* xof_given = nullptr;
};

// All pointers are device pointers; n handshakes processed as one chunk
// (the caller splits large batches).  Return hipError_t.
hipError_t mlkem_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins,
                         void* scratch, const Streams& st);
hipError_t mlkem_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                        const uint8_t* coins, int32_t* status, void* scratch, const Streams& st);
hipError_t mlkem_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk,
                        void* scratch, const Streams& st);

hipError_t frodo_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins,
                         void* scratch, const Streams& st);
hipError_t frodo_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                        const uint8_t* coins, void* scratch, const Streams& st);
hipError_t frodo_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk,
                        void* scratch, const Streams& st);

// HQC: decaps writes status[i] = -1 when the re-encryption check fails (ss = K(sigma || ct) is
// still written), the OQS_KEM_decaps return of liboqs; status may be NULL.
hipError_t hqc_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch,
                       const Streams& st);
hipError_t hqc_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins,
                      void* scratch, const Streams& st);
hipError_t hqc_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, int32_t* status,
                      void* scratch, const Streams& st);
// Fixed-weight supports from n vectors of random words r[n][w] (kind 0: w = the key weight,
// 1: w = the encryption weight w_r = w_e): sup_i = i + floor(r_i (n - i) / 2^32), deduplicated.
hipError_t hqc_supports(const AlgInfo& a, int kind, size_t n, const uint32_t* r, uint32_t* sup, hipStream_t st);

// SHAKE256("qrk-bench" || LE64(seed) || LE64(first + i), len) for i < n, len <= 136.
hipError_t bench_coins(size_t n, size_t len, uint64_t seed, uint64_t first, uint8_t* out, hipStream_t st);

// out_i = SHA3-256(a_i || b_i) (32 B per record); b may be NULL with bl = 0.
hipError_t digest_rows(size_t n, const uint8_t* a, size_t al, const uint8_t* b, size_t bl, uint8_t* out,
                       hipStream_t st);

// Flip one bit of ct_i for the indices selected by SHAKE256-derived Bernoulli(1/2)
// (bench config 5).  mode: 0 none, 1 all, 2 mixed.
hipError_t tamper_ciphertexts(size_t n, size_t ctlen, uint64_t seed, int mode, uint8_t* ct, hipStream_t st);

// HKDF-SHA256 (RFC 5869), one lane per key (hkdf.hip).  info_off (n+1 offsets) may be
// NULL, then every key uses info[0 .. info_len).  L <= 8160.
hipError_t hkdf_sha256(size_t n, const uint8_t* ikm, size_t ikm_len, size_t ikm_stride, const uint8_t* salt,
                       size_t salt_len, const uint8_t* info, const uint64_t* info_off, size_t info_len, size_t L,
                       uint8_t* okm, size_t okm_stride, hipStream_t st);
// agree_i = (a_i == b_i), len bytes each
hipError_t keys_equal(size_t n, const uint8_t* a, const uint8_t* b, size_t len, int32_t* agree, hipStream_t st);

// Standard base64 (RFC 4648, '=' padding) of n records of L bytes -> [n][4 ceil(L/3)] chars,
// and strict decoding back (status[i] = -1 for a malformed record; caller zeroes status).
hipError_t base64_encode(size_t n, const uint8_t* in, size_t L, uint8_t* out, hipStream_t st);
hipError_t base64_decode(size_t n, const uint8_t* in, size_t L, uint8_t* out, int32_t* status, hipStream_t st);

}  // namespace qrk
