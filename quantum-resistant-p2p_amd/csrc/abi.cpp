// C ABI of libqrkem.so (declared in include/qrkem.h).
//
// Part 1 mirrors the liboqs entry points bound by the reference's ctypes
// wrapper (quantum_resistant_p2p/vendor/oqs.py:192-198, 271, 318, 348, 372,
// 386-390, 397, 406-411); each single-shot call is a batch of one on the GPU.
// Part 2 is the batched device API.  There is no CPU fallback: with no HIP
// device every KEM call returns OQS_ERROR and qrk_last_error() says why.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qrkem.h"
#include "qrkem_internal.h"

// -DQRK_HOST_TRACE=1 (tools/build_variant.sh builds only): steady-clock stamps at the phases of a
// single-shot call, read by qrk_dbg_host_trace (tools/host_trace.py)
#ifndef QRK_HOST_TRACE
#define QRK_HOST_TRACE 0
#endif
#if QRK_HOST_TRACE
static long long g_host_trace[16];
#define HT(i) (g_host_trace[i] = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count())
extern "C" int qrk_dbg_host_trace(long long* out) {
  memcpy(out, g_host_trace, sizeof(g_host_trace));
  return 0;
}
#else
#define HT(i) ((void)0)
#endif

namespace qrk {

// ------------------------------------------------------------------ algorithm table
static AlgInfo ALGS[] = {
    // name, family, level, k/n, pk, sk, ct, ss, kp coins, enc coins, aes, enabled
    {"ML-KEM-512", Family::MLKEM, 1, 2, 800, 1632, 768, 32, 64, 32, false, true},
    {"ML-KEM-768", Family::MLKEM, 3, 3, 1184, 2400, 1088, 32, 64, 32, false, true},
    {"ML-KEM-1024", Family::MLKEM, 5, 4, 1568, 3168, 1568, 32, 64, 32, false, true},
    {"FrodoKEM-640-AES", Family::FRODO, 1, 640, 9616, 19888, 9720, 16, 48, 16, true, true},
    {"FrodoKEM-640-SHAKE", Family::FRODO, 1, 640, 9616, 19888, 9720, 16, 48, 16, false, true},
    {"FrodoKEM-976-AES", Family::FRODO, 3, 976, 15632, 31296, 15744, 24, 64, 24, true, true},
    {"FrodoKEM-976-SHAKE", Family::FRODO, 3, 976, 15632, 31296, 15744, 24, 64, 24, false, true},
    {"FrodoKEM-1344-AES", Family::FRODO, 5, 1344, 21520, 43088, 21632, 32, 80, 32, true, true},
    {"FrodoKEM-1344-SHAKE", Family::FRODO, 5, 1344, 21520, 43088, 21632, 32, 80, 32, false, true},
    {"HQC-128", Family::HQC, 1, 128, 2249, 2305, 4433, 64, 96, 32, false, true},
    {"HQC-192", Family::HQC, 3, 192, 4522, 4586, 8978, 64, 104, 40, false, true},
    {"HQC-256", Family::HQC, 5, 256, 7245, 7317, 14421, 64, 112, 48, false, true},
};
static const int NALG = (int)(sizeof(ALGS) / sizeof(ALGS[0]));

// Names liboqs supports that this engine does not implement (listed so that
// OQS_KEM_alg_is_enabled answers 0 rather than the name being unknown, the
// distinction oqs.py:265-269 draws between MechanismNotEnabledError and
// MechanismNotSupportedError).  Every KEM the reference selects is implemented.
static const char* UNIMPLEMENTED[] = {nullptr};
static const int NUNIMPL = 0;

const AlgInfo* find_alg(const char* name) {
  if (!name) return nullptr;
  for (int i = 0; i < NALG; ++i)
    if (!strcmp(ALGS[i].name, name)) return &ALGS[i];
  return nullptr;
}
int alg_count() { return NALG; }
const AlgInfo* alg_at(int i) { return (i >= 0 && i < NALG) ? &ALGS[i] : nullptr; }

}  // namespace qrk

using namespace qrk;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
static int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
static int hip_fail(const char* what, hipError_t e) {
  return fail(std::string(what) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------------ kernel timing
namespace qrk {
thread_local KernelTimer* g_timer = nullptr;
thread_local hipError_t g_launch_err = hipSuccess;
}

// Pairs of HIP events recorded on the launch stream around every kernel; read
// back (after a synchronise) as per-kernel-name totals.
struct EventTimer : KernelTimer {
  struct Rec {
    const char* name;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t pending = nullptr;
  hipEvent_t take() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    // timing only: no system-scope release (an L2 writeback + invalidate per event, which cost
    // 5 % of an ML-KEM-768 2^20 bench step with one event pair per launch)
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
  }
  void before(const char*, hipStream_t st) override {
    pending = take();
    (void)hipEventRecord(pending, st);
  }
  void after(const char* name, hipStream_t st) override {
    hipEvent_t b = take();
    (void)hipEventRecord(b, st);
    recs.push_back({name, pending, b});
    pending = nullptr;
  }
  void reset() {
    for (auto& r : recs) pool.push_back(r.a), pool.push_back(r.b);
    recs.clear();
  }
  ~EventTimer() override {
    reset();
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

// ------------------------------------------------------------------ context
struct qrk_ctx {
  int device = 0;
  size_t chunk = 1 << 20;
  bool profiling = false;
  EventTimer timer;
  std::vector<std::pair<std::string, std::pair<double, uint64_t>>> profile;  // name -> (ms, launches)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  uint8_t* dstage = nullptr;  // device staging for host-pointer calls and generated coins
  size_t dstage_bytes = 0;
  uint8_t* hstage = nullptr;  // pinned host staging
  size_t hstage_bytes = 0;
  uint8_t* hs_scratch = nullptr;  // handshake driver: ephemeral sk / ss of one chunk
  size_t hs_scratch_bytes = 0;
  uint8_t* dio = nullptr;         // host-pointer calls: packed device inputs | outputs
  size_t dio_bytes = 0;
  uint8_t* hio = nullptr;         // ... and their pinned host mirror
  size_t hio_bytes = 0;
  uint8_t* hio_dev = nullptr;     // device mapping of hio (zero-copy small calls)
  uint32_t* hflag = nullptr;      // single-shot completion flag (fine-grained pinned) ...
  uint32_t* hflag_dev = nullptr;  // ... its device address
  uint32_t* kg_cnt = nullptr;     // multi-workgroup ML-KEM KeyGen arrival counters (zeroed at allocation)
  bool kg_dirty = false;          // a pipelined KeyGen failed: a straggler may have set a flag word
                                  // after the collector's reset, or stored scratch after its wipe
  bool kg_err_next = false;       // run_batch: hand the KeyGen error word (hflag[1]) to the next launch
  uint64_t* xof_keep_next = nullptr;        // run_batch: Streams::xof_keep / xof_given of the next
  const uint64_t* xof_given_next = nullptr;  // call (handshake driver, one chunk)
  uint32_t* fixc = nullptr;       // ML-KEM SampleNTT fix-up counters of chunks <= 2^15 (Streams::fixc)
  int fixp = 0;                   // the counter the next such chunk counts into
  bool fixc_dirty = false;        // a chunk's launches failed after the parity flip: re-zero both
  uint32_t ticket = 0;
  bool flag_next = false;         // run_batch: hand the flag to the next launch
  const uint8_t* hin_next = nullptr;  // ... and the public input's host copy (a by-value kernel argument)
  hipStream_t io_stream = nullptr;
  int streams = 0;            // 0: multi-role launches, 1: serial (one kernel per launch)
  hipEvent_t ev_last = nullptr;  // recorded at the end of the last call that used the scratch
  hipStream_t last_stream = nullptr;  // ... on this stream
  bool last_valid = false;
  hipEvent_t ev_up = nullptr;    // end of the OS-coin upload (run_batch)
  mutable std::mutex mu;
};

// Calls that use a context's scratch are ordered one after another whatever stream each runs
// on: the new call's stream waits, on the device, on the event the previous call recorded at its
// end.  (A device-pointer call on the caller's stream followed by a host-pointer call on the
// context's own I/O stream would otherwise let the second overwrite scratch the first is still
// reading.)  This is the only cross-stream dependency of the library: every kernel of one call
// runs on that call's stream, so a device-pointer call never blocks the host.
static int ctx_order(qrk_ctx* ctx, hipStream_t st) {
  if (!ctx->ev_last) {
    hipError_t e = hipEventCreateWithFlags(&ctx->ev_last, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail("hipEventCreate(last use)", e);
  }
  if (ctx->last_valid && ctx->last_stream != st) {  // same stream: already in order
    hipError_t e = hipStreamWaitEvent(st, ctx->ev_last, 0);
    if (e != hipSuccess) return hip_fail("hipStreamWaitEvent(last use)", e);
  }
  return 0;
}
// Host-side wait for the previous call's device work (before freeing or refilling buffers it reads).
static void ctx_quiesce(qrk_ctx* ctx) {
  if (ctx->last_valid) (void)hipEventSynchronize(ctx->ev_last);
}
// Records the end of this call on `st` on every exit path, including early error returns.
struct LastUse {
  qrk_ctx* ctx;
  hipStream_t st;
  ~LastUse() {
    if (hipEventRecord(ctx->ev_last, st) == hipSuccess) {
      ctx->last_valid = true;
      ctx->last_stream = st;
    }
  }
};

// Makes `device` current for the scope of one ABI call and restores the caller's current
// device on exit, so a call on a context of GPU 3 never leaves the calling thread (and the
// torch allocations that follow) switched to GPU 3.
struct DeviceGuard {
  int prev = -1;
  int set(int device) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) return fail("no HIP device available (libqrkem has no CPU path)");
    if (device < 0 || device >= count) return fail("invalid device index");
    if (prev < 0 && hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev == device) return 0;
    e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    return 0;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

static int grow_device(qrk_ctx* ctx, void** p, size_t* have, size_t need, hipStream_t st) {
  if (*have >= need) return 0;
  if (*p) {
    ctx_quiesce(ctx);
    (void)hipStreamSynchronize(st);
    (void)hipMemset(*p, 0, *have);  // the old buffer may hold secret intermediates
    (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
  }
  hipError_t e = hipMalloc(p, need);
  if (e != hipSuccess) return hip_fail("hipMalloc", e);
  *have = need;
  return 0;
}

static int grow_pinned(uint8_t** p, size_t* have, size_t need) {
  if (*have >= need) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *have = 0;
  hipError_t e = hipHostMalloc((void**)p, need, hipHostMallocDefault);
  if (e != hipSuccess) return hip_fail("hipHostMalloc", e);
  *have = need;
  return 0;
}


static int os_random(uint8_t* out, size_t n) {
  while (n) {
    ssize_t r = getrandom(out, n, 0);
    if (r < 0) return fail("getrandom failed");
    out += r;
    n -= (size_t)r;
  }
  return 0;
}

static size_t scratch_for(const AlgInfo& a, size_t chunk) {
  switch (a.family) {
    case Family::MLKEM: return mlkem_scratch_bytes(a, chunk);
    case Family::FRODO: return frodo_scratch_bytes(a, chunk);
    default: return hqc_scratch_bytes(a, chunk);
  }
}

static hipError_t cleanse_records(const AlgInfo& a, size_t n, void* scratch, hipStream_t st) {
  switch (a.family) {
    case Family::MLKEM: return mlkem_cleanse(a, n, scratch, st);
    case Family::FRODO: return frodo_cleanse(a, n, scratch, st);
    default: return hqc_cleanse(a, n, scratch, st);
  }
}

static const AlgInfo* resolve(const char* alg) {
  const AlgInfo* a = find_alg(alg);
  if (!a) {
    for (int i = 0; alg && i < NUNIMPL; ++i)
      if (!strcmp(UNIMPLEMENTED[i], alg)) {
        fail(std::string("KEM not enabled in this build: ") + alg);
        return nullptr;
      }
    fail(std::string("unsupported KEM: ") + (alg ? alg : "(null)"));
    return nullptr;
  }
  if (!a->enabled) {
    fail(std::string("KEM not enabled in this build: ") + alg);
    return nullptr;
  }
  return a;
}

enum class Op { KEYPAIR, ENCAPS, DECAPS };

// FrodoKEM scratch is 0.14-0.53 MB per handshake, HQC's 9-24 KB: their chunks are capped so
// scratch stays near QRK_SCRATCH_GIB (48 GiB of the 288 GB HBM by default: a 2^16 FrodoKEM batch in
// one chunk, so the lane-per-handshake sponge kernels get a whole wave per SIMD)
#ifndef QRK_SCRATCH_GIB
#define QRK_SCRATCH_GIB 48
#endif
static size_t chunk_for(const qrk_ctx* ctx, const AlgInfo& a) {
  size_t cap = ctx->chunk;
  if (a.family != Family::MLKEM) {
    const size_t per_hs = scratch_for(a, 1024) / 1024 + 1;
    cap = std::min(cap, std::max<size_t>(4096, ((size_t)QRK_SCRATCH_GIB << 30) / per_hs / 64 * 64));
  }
  return cap;
}

// Routes QRK_LAUNCH timing to the context's timer for the scope's lifetime (nests).
struct TimerScope {
  KernelTimer* prev;
  explicit TimerScope(KernelTimer* t) : prev(g_timer) { g_timer = t; }
  ~TimerScope() { g_timer = prev; }
};

// Zeroes the device staging copy of OS-drawn coins when run_batch returns (these are
// the KeyGen seeds / Encaps messages, i.e. enough to rebuild the keys), stream-ordered after the
// kernels that read it.  The pinned host copy is wiped as soon as its upload has completed.
struct CoinWipe {
  qrk_ctx* ctx;
  hipStream_t st;
  size_t bytes = 0;
  ~CoinWipe() {
    if (bytes) (void)hipMemsetAsync(ctx->dstage, 0, bytes, st);
  }
};

// Core batched driver over device pointers, chunked.
static int run_batch(qrk_ctx* ctx, const AlgInfo& a, Op op, size_t n, uint8_t* o1, uint8_t* o2, const uint8_t* i1,
                     const uint8_t* i2, int32_t* status, hipStream_t st) {
  if (n == 0) return 0;
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  if (ctx_order(ctx, st)) return -1;
  LastUse last_use{ctx, st};
  // equal chunks (multiples of 64) rather than full chunks plus a small tail
  const size_t cap = chunk_for(ctx, a);
  const size_t nchunks = (n + cap - 1) / cap;
  const size_t chunk = std::min(cap, ((n + nchunks - 1) / nchunks + 63) & ~(size_t)63);
  if (grow_device(ctx, &ctx->scratch, &ctx->scratch_bytes, scratch_for(a, chunk), st)) return -1;
  // coins: NULL -> OS CSPRNG, uploaded to device staging
  const uint8_t* coins = (op == Op::KEYPAIR) ? i1 : (op == Op::ENCAPS ? i2 : nullptr);
  const size_t clen = (op == Op::KEYPAIR) ? a.kp_coins : a.enc_coins;
  // OS coins are KeyGen seeds / Encaps messages: wipe both staged copies on every exit path
  // (declared after last_use, so the device wipe is queued before the call's end event)
  CoinWipe coin_wipe{ctx, st};
  if (op != Op::DECAPS && coins == nullptr) {
    // The one host wait of the device-pointer API: the pinned copy of the coins is wiped as soon
    // as it has reached the device, so the call returns after the upload (which the stream
    // orders behind its earlier work), not after the kernels.
    const size_t bytes = n * clen;
    if (grow_pinned(&ctx->hstage, &ctx->hstage_bytes, bytes)) return -1;
    if (grow_device(ctx, (void**)&ctx->dstage, &ctx->dstage_bytes, bytes, st)) return -1;
    if (!ctx->ev_up) {
      hipError_t e = hipEventCreateWithFlags(&ctx->ev_up, hipEventDisableTiming);
      if (e != hipSuccess) return hip_fail("hipEventCreate(upload)", e);
    }
    if (os_random(ctx->hstage, bytes)) return -1;
    coin_wipe.bytes = bytes;
    hipError_t e = hipMemcpyAsync(ctx->dstage, ctx->hstage, bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_up, st);
    if (e == hipSuccess) e = hipEventSynchronize(ctx->ev_up);
    OQS_MEM_cleanse(ctx->hstage, bytes);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync(coins)", e);
    coins = ctx->dstage;
  }
  Streams S;
  S.main = st;
  // streams == 1: the documented serial schedule (one kernel per launch: per-kernel timings in
  // isolation, qrkem.h); otherwise independent kernels of one operation share launches
  S.serial = ctx->streams == 1;
  if (ctx->flag_next) {
    S.done = ctx->hflag_dev;
    S.ticket = ctx->ticket;
    S.host_in1 = ctx->hin_next;
  }
  if (a.family == Family::MLKEM && op == Op::KEYPAIR && n <= mlkem_kg_multi_max()) {
    if (!ctx->kg_cnt) {
      hipError_t e = hipMalloc((void**)&ctx->kg_cnt, mlkem_kg_flag_words() * sizeof(uint32_t));
      if (e == hipSuccess) e = hipMemset(ctx->kg_cnt, 0, mlkem_kg_flag_words() * sizeof(uint32_t));
      if (e != hipSuccess) return hip_fail("hipMalloc(kg_cnt)", e);
    }
    if (ctx->kg_dirty) {  // stream-ordered behind the failed call's kernel
      hipError_t e = hipMemsetAsync(ctx->kg_cnt, 0, mlkem_kg_flag_words() * sizeof(uint32_t), st);
      if (e == hipSuccess && ctx->scratch)
        e = hipMemsetAsync(ctx->scratch, 0, std::min(ctx->scratch_bytes, mlkem_kg_scratch_bytes()), st);
      if (e != hipSuccess) return hip_fail("hipMemsetAsync(kg_cnt)", e);
      ctx->kg_dirty = false;
    }
    S.kg_cnt = ctx->kg_cnt;
    if (ctx->kg_err_next) S.kg_err = ctx->hflag_dev + 1;
  }
  if (a.family == Family::MLKEM && n <= chunk && n > mlkem_small_max()) {
    S.xof_keep = op == Op::KEYPAIR ? ctx->xof_keep_next : nullptr;
    S.xof_given = op == Op::DECAPS ? ctx->xof_given_next : nullptr;
  }
  if (a.family == Family::MLKEM && op != Op::KEYPAIR) {
    if (!ctx->fixc) {
      hipError_t e = hipMalloc((void**)&ctx->fixc, 2 * sizeof(uint32_t));
      if (e == hipSuccess) e = hipMemset(ctx->fixc, 0, 2 * sizeof(uint32_t));
      if (e != hipSuccess) return hip_fail("hipMalloc(fixc)", e);
    }
    if (ctx->fixc_dirty) {
      const hipError_t e = hipMemsetAsync(ctx->fixc, 0, 2 * sizeof(uint32_t), st);
      if (e != hipSuccess) return hip_fail("hipMemsetAsync(fixc)", e);
      ctx->fixc_dirty = false;
    }
    S.fixc = ctx->fixc;
    S.fixp = &ctx->fixp;
  }
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  HT(3);
  for (size_t off = 0; off < n; off += chunk) {
    const size_t m = std::min(chunk, n - off);
    hipError_t e = hipSuccess;
    g_launch_err = hipSuccess;
    (void)hipGetLastError();  // clear a stale error state (e.g. a caller's hipErrorNotReady query)
    if (a.family == Family::MLKEM) {
      switch (op) {
        case Op::KEYPAIR:
          e = mlkem_keypair(a, m, o1 + off * a.pk, o2 + off * a.sk, coins + off * clen, ctx->scratch, S);
          break;
        case Op::ENCAPS:
          e = mlkem_encaps(a, m, o1 + off * a.ct, o2 + off * a.ss, i1 + off * a.pk, coins + off * clen,
                           status ? status + off : nullptr, ctx->scratch, S);
          break;
        case Op::DECAPS:
          if (status) e = hipMemsetAsync(status + off, 0, m * sizeof(int32_t), st);
          if (e == hipSuccess)
            e = mlkem_decaps(a, m, o1 + off * a.ss, i1 + off * a.ct, i2 + off * a.sk, ctx->scratch, S);
          break;
      }
    } else if (a.family == Family::HQC) {
      switch (op) {
        case Op::KEYPAIR:
          e = hqc_keypair(a, m, o1 + off * a.pk, o2 + off * a.sk, coins + off * clen, ctx->scratch, S);
          break;
        case Op::ENCAPS:
          // HQC encapsulation has no public-key validity check: status is always 0
          if (status) e = hipMemsetAsync(status + off, 0, m * sizeof(int32_t), st);
          if (e == hipSuccess)
            e = hqc_encaps(a, m, o1 + off * a.ct, o2 + off * a.ss, i1 + off * a.pk, coins + off * clen, ctx->scratch,
                           S);
          break;
        case Op::DECAPS:
          e = hqc_decaps(a, m, o1 + off * a.ss, i1 + off * a.ct, i2 + off * a.sk, status ? status + off : nullptr,
                         ctx->scratch, S);
          break;
      }
    } else {
      switch (op) {
        case Op::KEYPAIR:
          e = frodo_keypair(a, m, o1 + off * a.pk, o2 + off * a.sk, coins + off * clen, ctx->scratch, S);
          break;
        case Op::ENCAPS:
          // FrodoKEM encapsulation has no public-key validity check: status is always 0
          if (status) e = hipMemsetAsync(status + off, 0, m * sizeof(int32_t), st);
          if (e == hipSuccess)
            e = frodo_encaps(a, m, o1 + off * a.ct, o2 + off * a.ss, i1 + off * a.pk, coins + off * clen,
                             ctx->scratch, S);
          break;
        case Op::DECAPS:
          if (status) e = hipMemsetAsync(status + off, 0, m * sizeof(int32_t), st);
          if (e == hipSuccess)
            e = frodo_decaps(a, m, o1 + off * a.ss, i1 + off * a.ct, i2 + off * a.sk, ctx->scratch, S);
          break;
      }
    }
    HT(4);
    if (e == hipSuccess) e = g_launch_err;
    if (e != hipSuccess) {
      ctx->fixc_dirty = S.fixc != nullptr;  // the counters' zero-between-calls invariant is unknown now
      return hip_fail("kernel launch", e);
    }
    // key material of this chunk (seeds, m', K', Kbar, ...) does not outlive the call
    e = cleanse_records(a, m, ctx->scratch, st);
    if (e != hipSuccess) return hip_fail("hipMemsetAsync(cleanse)", e);
  }
  return 0;
}

// The single-shot completion flag: one word of fine-grained (coherent) pinned memory.
static int flag_ready(qrk_ctx* ctx) {
  if (ctx->hflag_dev) return 0;
  hipError_t e = hipHostMalloc((void**)&ctx->hflag, 64, hipHostMallocCoherent);
  if (e != hipSuccess) return hip_fail("hipHostMalloc(flag)", e);
  *ctx->hflag = 0;
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, ctx->hflag, 0);
  if (e != hipSuccess) return hip_fail("hipHostGetDevicePointer(flag)", e);
  ctx->hflag_dev = (uint32_t*)d;
  return 0;
}

// Zero-copy host call (see run_batch_host): inputs | outputs packed in the pinned mirror, which
// the kernel addresses through its device mapping.
static int run_small_host(qrk_ctx* ctx, const AlgInfo& a, Op op, size_t n, uint8_t* o1, uint8_t* o2,
                          const uint8_t* i1, const uint8_t* i2, int32_t* status, size_t l_o1, size_t l_o2,
                          size_t l_i1, size_t l_i2, hipStream_t st) {
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t b_i1 = al(n * l_i1), b_i2 = al(n * l_i2), b_o1 = al(n * l_o1), b_o2 = al(n * l_o2);
  const size_t b_st = al(n * sizeof(int32_t)), total = b_i1 + b_i2 + b_o1 + b_o2 + b_st;
  if (ctx->hio_bytes < total) {
    ctx_quiesce(ctx);
    if (ctx->hio) OQS_MEM_cleanse(ctx->hio, ctx->hio_bytes);
    if (grow_pinned(&ctx->hio, &ctx->hio_bytes, total)) return -1;
    ctx->hio_dev = nullptr;
  }
  if (!ctx->hio_dev) {
    void* d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, ctx->hio, 0);
    if (e != hipSuccess) return hip_fail("hipHostGetDevicePointer", e);
    ctx->hio_dev = (uint8_t*)d;
  }
  uint8_t* h = ctx->hio;
  const size_t o_i2 = b_i1, o_o1 = b_i1 + b_i2, o_o2 = o_o1 + b_o1, o_st = o_o2 + b_o2;
  // inputs (coins the caller did not supply come from the OS CSPRNG)
  if (l_i1) {
    if (i1) memcpy(h, i1, n * l_i1);
    else if (os_random(h, n * l_i1)) return -1;
  }
  if (l_i2) {
    if (i2) memcpy(h + o_i2, i2, n * l_i2);
    else if (os_random(h + o_i2, n * l_i2)) return -1;
  }
  memset(h + o_st, 0, n * sizeof(int32_t));
  HT(2);
  uint8_t* d = ctx->hio_dev;
  // n == 1: the kernel stores a ticket in fine-grained pinned memory once its outputs are visible,
  // and the host spins on it (about 4 us sooner than hipStreamSynchronize wakes up)
  const bool spin = n == 1 && flag_ready(ctx) == 0;
  // ML-KEM KeyGen: the pipelined kernel's error word, hflag[1] (the flag's 64-byte line)
  const bool kg_err = op == Op::KEYPAIR && n <= mlkem_kg_multi_max() && flag_ready(ctx) == 0;
  if (kg_err) {
    __atomic_store_n(ctx->hflag + 1, 0u, __ATOMIC_RELEASE);
    ctx->kg_err_next = true;
  }
  if (spin) {
    ctx->ticket = ctx->ticket + 1 ? ctx->ticket + 1 : 1;
    ctx->flag_next = true;
    // the public input (Encaps pk, Decaps c) may travel as a kernel argument; KeyGen's coins never
    ctx->hin_next = (op != Op::KEYPAIR && l_i1) ? h : nullptr;
  }
  // ML-KEM decapsulation reports no status (implicit rejection): only encapsulation writes it
  int rc = run_batch(ctx, a, op, n, d + o_o1, l_o2 ? d + o_o2 : nullptr, l_i1 ? d : nullptr, l_i2 ? d + o_i2 : nullptr,
                     (status && op == Op::ENCAPS) ? (int32_t*)(d + o_st) : nullptr, st);
  HT(5);
  ctx->flag_next = false;
  ctx->hin_next = nullptr;
  ctx->kg_err_next = false;
  hipError_t e = hipSuccess;
  if (!rc && spin) {
    // bounded spin; a kernel that never stores the ticket (a launch or execution error) falls
    // back to the stream synchronise, which reports it
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    for (unsigned k = 0;; ++k) {
      if (__atomic_load_n(ctx->hflag, __ATOMIC_ACQUIRE) == ctx->ticket) {
        seen = true;
        break;
      }
      if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) break;
    }
    HT(6);
    if (!seen) e = hipStreamSynchronize(st);
  } else if (!rc) {
    e = hipStreamSynchronize(st);
  }
  if (!rc && e != hipSuccess) rc = hip_fail("kernel execution", e);
  // the collector stores the error word before the ticket (or the kernel's end, which the stream
  // synchronise waited for)
  if (!rc && kg_err && __atomic_load_n(ctx->hflag + 1, __ATOMIC_ACQUIRE) != 0)
    rc = fail("ML-KEM KeyGen: keygen hand-off timeout (a bounded cross-workgroup wait expired)");
  if (rc && kg_err) ctx->kg_dirty = true;  // re-zeroed (flags, scratch) before the next KeyGen launch
  if (!rc) {
    memcpy(o1, h + o_o1, n * l_o1);
    if (l_o2) memcpy(o2, h + o_o2, n * l_o2);
    if (status) memcpy(status, h + o_st, n * sizeof(int32_t));
  }
  if (rc) (void)hipStreamSynchronize(st);  // nothing may still read or write the mirror
  if (rc && ctx->kg_dirty && ctx->kg_cnt) {
    // wipe the secret scratch a straggler may have written after the collector's wipe now, not at
    // the next KeyGen (run_batch re-zeroes again if this fails)
    hipError_t w = hipMemsetAsync(ctx->kg_cnt, 0, mlkem_kg_flag_words() * sizeof(uint32_t), st);
    if (w == hipSuccess && ctx->scratch)
      w = hipMemsetAsync(ctx->scratch, 0, std::min(ctx->scratch_bytes, mlkem_kg_scratch_bytes()), st);
    if (w == hipSuccess) w = hipStreamSynchronize(st);
    if (w == hipSuccess) ctx->kg_dirty = false;
  }
  OQS_MEM_cleanse(h, total);  // coins, secret keys and shared secrets do not outlive the call
  HT(7);
  return rc;
}

// Host-pointer wrapper: stage inputs, run, copy outputs back, synchronise.  The context
// keeps a device I/O buffer, a pinned host mirror and its own stream, so a call is one
// packed H2D copy, the kernels, one packed D2H copy and one synchronise (the reference's
// one-handshake-per-call pattern, oqs.py:318, 348, 372, pays no allocation per call).
static int run_batch_host(qrk_ctx* ctx, const AlgInfo& a, Op op, size_t n, uint8_t* o1, uint8_t* o2,
                          const uint8_t* i1, const uint8_t* i2, int32_t* status) {
  if (n == 0) return 0;
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  // Small ML-KEM batches (one launch per operation, the reference's single-shot calls) run
  // zero-copy: the kernel reads its inputs from and writes its outputs to the pinned mirror, and
  // coins are drawn straight into it, so a call is one launch and one synchronise.
  const bool zc = a.family == Family::MLKEM && n <= mlkem_small_max();
  size_t l_o1, l_o2, l_i1, l_i2;
  switch (op) {
    case Op::KEYPAIR: l_o1 = a.pk, l_o2 = a.sk, l_i1 = (i1 || zc) ? a.kp_coins : 0, l_i2 = 0; break;
    case Op::ENCAPS: l_o1 = a.ct, l_o2 = a.ss, l_i1 = a.pk, l_i2 = (i2 || zc) ? a.enc_coins : 0; break;
    default: l_o1 = a.ss, l_o2 = 0, l_i1 = a.ct, l_i2 = a.sk; break;
  }
  const size_t l_st = status ? sizeof(int32_t) : 0;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  // inputs first (one H2D), then outputs (one D2H)
  const size_t b_i1 = al(n * l_i1), b_i2 = al(n * l_i2), b_o1 = al(n * l_o1), b_o2 = al(n * l_o2),
               b_st = al(n * l_st);
  const size_t in_bytes = b_i1 + b_i2, out_bytes = b_o1 + b_o2 + b_st;
  if (!ctx->io_stream) {
    hipError_t e = hipStreamCreateWithFlags(&ctx->io_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail("hipStreamCreate(io)", e);
  }
  hipStream_t st = ctx->io_stream;
  if (zc) return run_small_host(ctx, a, op, n, o1, o2, i1, i2, status, l_o1, l_o2, l_i1, l_i2, st);
  if (grow_device(ctx, (void**)&ctx->dio, &ctx->dio_bytes, in_bytes + out_bytes, st)) return -1;
  if (ctx->hio_bytes < in_bytes + out_bytes) ctx->hio_dev = nullptr;  // reallocated below
  if (grow_pinned(&ctx->hio, &ctx->hio_bytes, in_bytes + out_bytes)) return -1;
  uint8_t *d_i1 = ctx->dio, *d_i2 = d_i1 + b_i1, *d_o1 = d_i2 + b_i2, *d_o2 = d_o1 + b_o1, *d_st = d_o2 + b_o2;
  uint8_t* h = ctx->hio;
  if (l_i1) memcpy(h, i1, n * l_i1);
  if (l_i2) memcpy(h + b_i1, i2, n * l_i2);
  hipError_t e = in_bytes ? hipMemcpyAsync(ctx->dio, h, in_bytes, hipMemcpyHostToDevice, st) : hipSuccess;
  if (e != hipSuccess) return hip_fail("hipMemcpyAsync(H2D)", e);
  int rc = run_batch(ctx, a, op, n, d_o1, l_o2 ? d_o2 : nullptr, l_i1 ? d_i1 : nullptr, l_i2 ? d_i2 : nullptr,
                     status ? (int32_t*)d_st : nullptr, st);
  if (rc) return rc;
  uint8_t* ho = h + in_bytes;
  e = hipMemcpyAsync(ho, d_o1, out_bytes, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail("kernel execution / D2H", e);
  memcpy(o1, ho, n * l_o1);
  if (l_o2) memcpy(o2, ho + b_o1, n * l_o2);
  if (status) memcpy(status, ho + b_o1 + b_o2, n * l_st);
  // the staged copies of secret keys, coins and shared secrets do not outlive the call:
  // KeyGen (coins in, sk out), Encaps (coins in, ss out), Decaps (sk in, ss out)
  struct Span {
    size_t off, len;
  };
  const Span sec[2] = {op == Op::KEYPAIR   ? Span{0, n * l_i1}
                       : op == Op::ENCAPS  ? Span{b_i1, n * l_i2}
                                           : Span{b_i1, n * l_i2},
                       op == Op::KEYPAIR ? Span{in_bytes + b_o1, n * l_o2}
                       : op == Op::ENCAPS ? Span{in_bytes + b_o1, n * l_o2}
                                          : Span{in_bytes, n * l_o1}};
  for (const Span& z : sec) {
    if (!z.len) continue;
    OQS_MEM_cleanse(h + z.off, z.len);
    (void)hipMemsetAsync(ctx->dio + z.off, 0, z.len, st);
  }
  return 0;
}

// ------------------------------------------------------------------ default context (single-shot API)
static std::mutex g_default_mu;
static qrk_ctx* g_default = nullptr;

static qrk_ctx* default_ctx() {
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (!g_default) {
    g_default = new qrk_ctx();
    const char* dev = getenv("QRK_DEVICE");
    g_default->device = dev ? atoi(dev) : 0;
    g_default->chunk = 1 << 12;
  }
  return g_default;
}

static OQS_STATUS single(const AlgInfo& a, Op op, uint8_t* o1, uint8_t* o2, const uint8_t* i1, const uint8_t* i2) {
  HT(0);
  qrk_ctx* ctx = default_ctx();
  std::lock_guard<std::mutex> lk(ctx->mu);
  int32_t status = 0;
  HT(1);
  int rc = run_batch_host(ctx, a, op, 1, o1, o2, i1, i2, op == Op::KEYPAIR ? nullptr : &status);
  HT(9);
  // ML-KEM encaps: the FIPS 203 modulus check; HQC decaps: liboqs returns OQS_ERROR when the
  // re-encryption check fails (the shared secret K(sigma || ct) is still written)
  if (rc == 0 && status != 0)
    rc = fail(op == Op::ENCAPS ? "encapsulation key failed the FIPS 203 modulus check"
                               : "ciphertext rejected by the re-encryption check");
  return rc == 0 ? OQS_SUCCESS : OQS_ERROR;
}

// per-algorithm callbacks stored in OQS_KEM (liboqs semantics: no kem argument)
template <int I>
static OQS_STATUS cb_keypair(uint8_t* pk, uint8_t* sk) {
  return single(ALGS[I], Op::KEYPAIR, pk, sk, nullptr, nullptr);
}
template <int I>
static OQS_STATUS cb_encaps(uint8_t* ct, uint8_t* ss, const uint8_t* pk) {
  return single(ALGS[I], Op::ENCAPS, ct, ss, pk, nullptr);
}
template <int I>
static OQS_STATUS cb_decaps(uint8_t* ss, const uint8_t* ct, const uint8_t* sk) {
  return single(ALGS[I], Op::DECAPS, ss, nullptr, ct, sk);
}

template <int I>
static void fill_cbs(OQS_KEM* k, int idx) {
  if constexpr (I < (int)(sizeof(ALGS) / sizeof(ALGS[0]))) {
    if (idx == I) {
      k->keypair = cb_keypair<I>;
      k->encaps = cb_encaps<I>;
      k->decaps = cb_decaps<I>;
      return;
    }
    fill_cbs<I + 1>(k, idx);
  }
}

extern "C" {

// ------------------------------------------------------------------ Part 1: liboqs subset
void OQS_init(void) {}

const char* OQS_version(void) { return "0.12.0-qrkem-gfx950"; }

size_t OQS_KEM_alg_count(void) { return (size_t)(NALG + NUNIMPL); }

const char* OQS_KEM_alg_identifier(size_t i) {
  if (i < (size_t)NALG) return ALGS[i].name;
  if (i < (size_t)(NALG + NUNIMPL)) return UNIMPLEMENTED[i - NALG];
  return nullptr;
}

int OQS_KEM_alg_is_enabled(const char* method_name) {
  const AlgInfo* a = find_alg(method_name);
  return a && a->enabled ? 1 : 0;
}

OQS_KEM* OQS_KEM_new(const char* method_name) {
  const AlgInfo* a = find_alg(method_name);
  if (!a || !a->enabled) return nullptr;
  OQS_KEM* k = (OQS_KEM*)calloc(1, sizeof(OQS_KEM));
  if (!k) return nullptr;
  k->method_name = a->name;
  k->alg_version = a->family == Family::MLKEM   ? "FIPS203 (qrkem gfx950)"
                   : a->family == Family::FRODO ? "FrodoKEM round 3 (qrkem gfx950)"
                                                : "HQC 2023-04-30 (qrkem gfx950)";
  k->claimed_nist_level = (uint8_t)a->level;
  k->ind_cca = true;
  k->length_public_key = a->pk;
  k->length_secret_key = a->sk;
  k->length_ciphertext = a->ct;
  k->length_shared_secret = a->ss;
  fill_cbs<0>(k, (int)(a - ALGS));
  return k;
}

static const AlgInfo* alg_of(const OQS_KEM* kem) {
  if (!kem) {
    fail("null OQS_KEM");
    return nullptr;
  }
  return resolve(kem->method_name);
}

OQS_STATUS OQS_KEM_keypair(const OQS_KEM* kem, uint8_t* pk, uint8_t* sk) {
  const AlgInfo* a = alg_of(kem);
  return a ? single(*a, Op::KEYPAIR, pk, sk, nullptr, nullptr) : OQS_ERROR;
}
OQS_STATUS OQS_KEM_keypair_derand(const OQS_KEM* kem, uint8_t* pk, uint8_t* sk, const uint8_t* seed) {
  const AlgInfo* a = alg_of(kem);
  if (!a || !seed) return OQS_ERROR;
  return single(*a, Op::KEYPAIR, pk, sk, seed, nullptr);
}
OQS_STATUS OQS_KEM_encaps(const OQS_KEM* kem, uint8_t* ct, uint8_t* ss, const uint8_t* pk) {
  const AlgInfo* a = alg_of(kem);
  return a ? single(*a, Op::ENCAPS, ct, ss, pk, nullptr) : OQS_ERROR;
}
OQS_STATUS OQS_KEM_encaps_derand(const OQS_KEM* kem, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                                 const uint8_t* seed) {
  const AlgInfo* a = alg_of(kem);
  if (!a || !seed) return OQS_ERROR;
  return single(*a, Op::ENCAPS, ct, ss, pk, seed);
}
OQS_STATUS OQS_KEM_decaps(const OQS_KEM* kem, uint8_t* ss, const uint8_t* ct, const uint8_t* sk) {
  const AlgInfo* a = alg_of(kem);
  return a ? single(*a, Op::DECAPS, ss, nullptr, ct, sk) : OQS_ERROR;
}
void OQS_KEM_free(OQS_KEM* kem) { free(kem); }

// Empty signature registry (see include/qrkem.h)
size_t OQS_SIG_alg_count(void) { return 0; }
const char* OQS_SIG_alg_identifier(size_t) { return nullptr; }
int OQS_SIG_alg_is_enabled(const char*) { return 0; }
OQS_SIG* OQS_SIG_new(const char*) {
  fail("signatures are not implemented by libqrkem");
  return nullptr;
}
OQS_STATUS OQS_SIG_keypair(const OQS_SIG*, uint8_t*, uint8_t*) { return OQS_ERROR; }
OQS_STATUS OQS_SIG_sign(const OQS_SIG*, uint8_t*, size_t*, const uint8_t*, size_t, const uint8_t*) {
  return OQS_ERROR;
}
OQS_STATUS OQS_SIG_verify(const OQS_SIG*, const uint8_t*, size_t, const uint8_t*, size_t, const uint8_t*) {
  return OQS_ERROR;
}
void OQS_SIG_free(OQS_SIG*) {}

void OQS_MEM_cleanse(void* ptr, size_t len) {
  if (!ptr) return;
  volatile uint8_t* p = (volatile uint8_t*)ptr;
  while (len--) *p++ = 0;
}

// ------------------------------------------------------------------ Part 2: batched API
int qrk_ctx_create(qrk_ctx** out, int device) {
  if (!out) return fail("null out");
  *out = nullptr;
  DeviceGuard device_guard;
  if (device_guard.set(device)) return -1;
  qrk_ctx* c = new qrk_ctx();
  c->device = device;
  *out = c;
  return 0;
}

// Zero every buffer of the context that can hold keys or secret intermediates (device scratch,
// handshake scratch, device and pinned host staging).  Synchronous.
static void cleanse_all(qrk_ctx* ctx) {
  ctx_quiesce(ctx);
  if (ctx->scratch) (void)hipMemset(ctx->scratch, 0, ctx->scratch_bytes);
  if (ctx->hs_scratch) (void)hipMemset(ctx->hs_scratch, 0, ctx->hs_scratch_bytes);
  if (ctx->dio) (void)hipMemset(ctx->dio, 0, ctx->dio_bytes);
  if (ctx->dstage) (void)hipMemset(ctx->dstage, 0, ctx->dstage_bytes);
  (void)hipDeviceSynchronize();
  if (ctx->hio) OQS_MEM_cleanse(ctx->hio, ctx->hio_bytes);
  if (ctx->hstage) OQS_MEM_cleanse(ctx->hstage, ctx->hstage_bytes);
}

int qrk_ctx_cleanse(qrk_ctx* ctx) {
  if (!ctx) return fail("null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  cleanse_all(ctx);
  return 0;
}

void qrk_ctx_destroy(qrk_ctx* ctx) {
  if (!ctx) return;
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device) == 0) {
    (void)hipDeviceSynchronize();
    cleanse_all(ctx);
  }
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->hs_scratch) (void)hipFree(ctx->hs_scratch);
  if (ctx->dio) (void)hipFree(ctx->dio);
  if (ctx->hio) (void)hipHostFree(ctx->hio);
  if (ctx->hflag) (void)hipHostFree(ctx->hflag);
  if (ctx->io_stream) (void)hipStreamDestroy(ctx->io_stream);
  if (ctx->dstage) (void)hipFree(ctx->dstage);
  if (ctx->hstage) (void)hipHostFree(ctx->hstage);
  if (ctx->kg_cnt) (void)hipFree(ctx->kg_cnt);
  if (ctx->fixc) (void)hipFree(ctx->fixc);
  if (ctx->ev_up) (void)hipEventDestroy(ctx->ev_up);
  if (ctx->ev_last) (void)hipEventDestroy(ctx->ev_last);
  delete ctx;
}

int qrk_ctx_set_streams(qrk_ctx* ctx, int streams) {
  if (!ctx || streams < 0 || streams > 1) return fail("streams must be 0 (auto) or 1 (serial)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->streams = streams;
  return 0;
}

int qrk_ctx_set_chunk(qrk_ctx* ctx, size_t chunk) {
  if (!ctx || chunk == 0) return fail("bad chunk");
  std::lock_guard<std::mutex> lk(ctx->mu);  // chunk_for reads it under the lock
  ctx->chunk = (chunk + 63) & ~(size_t)63;
  return 0;
}

size_t qrk_ctx_scratch_bytes(const qrk_ctx* ctx) { return ctx ? ctx->scratch_bytes : 0; }

int qrk_ctx_staging_residue(qrk_ctx* ctx, uint64_t out[3]) {
  if (!ctx || !out) return fail("null argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  ctx_quiesce(ctx);
  out[0] = out[1] = out[2] = 0;
  for (size_t i = 0; i < ctx->hstage_bytes; ++i) out[0] += ctx->hstage[i] != 0;
  const void* src[2] = {ctx->dstage, ctx->scratch};
  const size_t len[2] = {ctx->dstage_bytes, std::min<size_t>(ctx->scratch_bytes, (size_t)64 << 20)};
  for (int b = 0; b < 2; ++b) {
    if (!len[b]) continue;
    std::vector<uint8_t> tmp(len[b]);
    hipError_t e = hipMemcpy(tmp.data(), src[b], len[b], hipMemcpyDeviceToHost);
    for (uint8_t x : tmp) out[1 + b] += x != 0;
    // the copy may hold expanded key material (PRF / CBD output, FrodoKEM S, HQC x, y): wipe it
    // before the heap gets it back
    OQS_MEM_cleanse(tmp.data(), tmp.size());
    if (e != hipSuccess) return hip_fail("hipMemcpy(staging residue)", e);
  }
  return 0;
}

// Tests only (not in qrkem.h): the workgroup of role `role` of the pipelined single-shot ML-KEM KeyGen
// (PRF item N = role < 2K, row r = role - 2K + 1) publishes its payload and flags 150 ms late, past
// every bounded wait (-1: off).  Process-wide.
extern "C" int qrk_dbg_kg_late(int role) {
  g_kg_dbg_late = role;
  return 0;
}

// Tests only (not in qrkem.h): batched ML-KEM Encaps / Decaps chunks of at most 2^15 handshakes fail
// right after the SampleNTT fix-up counter parity flip, before their first launch (0: off), and the
// context's two fix-up counter words and its parity read back (the re-zero path).
extern "C" int qrk_dbg_fail_after_flip(int on) {
  g_dbg_fail_after_flip = on;
  return 0;
}
extern "C" int qrk_dbg_fixc_words(qrk_ctx* ctx, uint32_t* out, int* parity) {
  if (!ctx || !out || !parity) return fail("null argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  ctx_quiesce(ctx);
  out[0] = out[1] = 0;
  *parity = ctx->fixp;
  if (!ctx->fixc) return 0;
  const hipError_t e = hipMemcpy(out, ctx->fixc, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : hip_fail("hipMemcpy(fixc)", e);
}

// Tests only (not in qrkem.h): nonzero words among the context's single-shot KeyGen flag / counter
// words, which must be zero between calls (after a failed pipelined KeyGen too).
extern "C" int qrk_dbg_kg_flags_residue(qrk_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return fail("null argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  ctx_quiesce(ctx);
  *out = 0;
  if (!ctx->kg_cnt) return 0;
  std::vector<uint32_t> tmp(mlkem_kg_flag_words());
  const hipError_t e = hipMemcpy(tmp.data(), ctx->kg_cnt, tmp.size() * sizeof(uint32_t), hipMemcpyDeviceToHost);
  for (uint32_t x : tmp) *out += x != 0;
  return e == hipSuccess ? 0 : hip_fail("hipMemcpy(kg flags)", e);
}

// Tests only (not in qrkem.h): nonzero bytes left in the ML-KEM per-handshake records of a chunk
// of n handshakes (mlkem_cleanse wipes them after every chunk).
extern "C" int qrk_dbg_mlkem_records_residue(qrk_ctx* ctx, const char* alg, size_t n, uint64_t* out) {
  if (!ctx || !out) return fail("null argument");
  const AlgInfo* a = find_alg(alg);
  if (!a || a->family != Family::MLKEM) return fail("not an ML-KEM algorithm");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  ctx_quiesce(ctx);
  size_t off = 0, bytes = 0;
  mlkem_records_span(*a, (std::min(n, chunk_for(ctx, *a)) + 63) & ~(size_t)63, &off, &bytes);
  if (off + bytes > ctx->scratch_bytes) return fail("the context's scratch does not cover that chunk");
  std::vector<uint8_t> tmp(bytes);
  const hipError_t e = hipMemcpy(tmp.data(), (const char*)ctx->scratch + off, bytes, hipMemcpyDeviceToHost);
  *out = 0;
  for (uint8_t x : tmp) *out += x != 0;
  OQS_MEM_cleanse(tmp.data(), tmp.size());
  return e == hipSuccess ? 0 : hip_fail("hipMemcpy(records residue)", e);
}

size_t qrk_ctx_effective_chunk(const qrk_ctx* ctx, const char* alg) {
  const AlgInfo* a = find_alg(alg);
  if (!ctx || !a) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return chunk_for(ctx, *a);
}

int qrk_ctx_profile(qrk_ctx* ctx, int enable) {
  if (!ctx) return fail("null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->timer.reset();
  ctx->profile.clear();
  ctx->profiling = enable != 0;
  return 0;
}

int qrk_ctx_profile_collect(qrk_ctx* ctx) {
  if (!ctx) return fail("null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (auto& r : ctx->timer.recs) {
    hipError_t e = hipEventSynchronize(r.b);
    if (e != hipSuccess) return hip_fail("hipEventSynchronize", e);
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess) return hip_fail("hipEventElapsedTime", e);
    auto it = std::find_if(ctx->profile.begin(), ctx->profile.end(),
                           [&](const auto& p) { return p.first == r.name; });
    if (it == ctx->profile.end()) {
      ctx->profile.push_back({r.name, {ms, 1}});
    } else {
      it->second.first += ms;
      it->second.second += 1;
    }
  }
  ctx->timer.reset();
  return (int)ctx->profile.size();
}

int qrk_ctx_profile_get(qrk_ctx* ctx, int i, const char** name, double* total_ms, uint64_t* launches) {
  if (!ctx || i < 0 || i >= (int)ctx->profile.size()) return fail("profile index out of range");
  *name = ctx->profile[i].first.c_str();
  *total_ms = ctx->profile[i].second.first;
  *launches = ctx->profile[i].second.second;
  return 0;
}

int qrk_kem_sizes(const char* alg, size_t out[6]) {
  const AlgInfo* a = find_alg(alg);
  if (!a) return fail(std::string("unsupported KEM: ") + (alg ? alg : "(null)"));
  out[0] = a->pk, out[1] = a->sk, out[2] = a->ct, out[3] = a->ss, out[4] = a->kp_coins, out[5] = a->enc_coins;
  return 0;
}

#define QRK_RESOLVE(ctx, alg)                \
  if (!(ctx)) return fail("null context");   \
  const AlgInfo* a = resolve(alg);           \
  if (!a) return -1;                         \
  std::lock_guard<std::mutex> lk((ctx)->mu);

int qrk_kem_keypair_batch(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins,
                          void* stream) {
  QRK_RESOLVE(ctx, alg);
  return run_batch(ctx, *a, Op::KEYPAIR, n, pk, sk, coins, nullptr, nullptr, (hipStream_t)stream);
}
int qrk_kem_encaps_batch(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                         const uint8_t* coins, int32_t* status, void* stream) {
  QRK_RESOLVE(ctx, alg);
  return run_batch(ctx, *a, Op::ENCAPS, n, ct, ss, pk, coins, status, (hipStream_t)stream);
}
int qrk_kem_decaps_batch(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk,
                         void* stream) {
  QRK_RESOLVE(ctx, alg);
  return run_batch(ctx, *a, Op::DECAPS, n, ss, nullptr, ct, sk, nullptr, (hipStream_t)stream);
}
int qrk_kem_decaps_batch_status(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ss, const uint8_t* ct,
                                const uint8_t* sk, int32_t* status, void* stream) {
  QRK_RESOLVE(ctx, alg);
  return run_batch(ctx, *a, Op::DECAPS, n, ss, nullptr, ct, sk, status, (hipStream_t)stream);
}
int qrk_kem_keypair_batch_host(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* pk, uint8_t* sk,
                               const uint8_t* coins) {
  QRK_RESOLVE(ctx, alg);
  return run_batch_host(ctx, *a, Op::KEYPAIR, n, pk, sk, coins, nullptr, nullptr);
}
int qrk_kem_encaps_batch_host(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                              const uint8_t* coins, int32_t* status) {
  QRK_RESOLVE(ctx, alg);
  return run_batch_host(ctx, *a, Op::ENCAPS, n, ct, ss, pk, coins, status);
}
int qrk_kem_decaps_batch_host(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ss, const uint8_t* ct,
                              const uint8_t* sk) {
  QRK_RESOLVE(ctx, alg);
  return run_batch_host(ctx, *a, Op::DECAPS, n, ss, nullptr, ct, sk, nullptr);
}
int qrk_kem_decaps_batch_status_host(qrk_ctx* ctx, const char* alg, size_t n, uint8_t* ss, const uint8_t* ct,
                                     const uint8_t* sk, int32_t* status) {
  QRK_RESOLVE(ctx, alg);
  return run_batch_host(ctx, *a, Op::DECAPS, n, ss, nullptr, ct, sk, status);
}

int qrk_bench_coins(qrk_ctx* ctx, size_t n, size_t len, uint64_t seed, uint64_t first, uint8_t* out, void* stream) {
  if (!ctx) return fail("null context");
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  hipError_t e = bench_coins(n, len, seed, first, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("bench_coins", e);
}

int qrk_tamper(qrk_ctx* ctx, size_t n, size_t ctlen, uint64_t seed, int mode, uint8_t* ct, void* stream) {
  if (!ctx) return fail("null context");
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  hipError_t e = tamper_ciphertexts(n, ctlen, seed, mode, ct, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("tamper", e);
}

int qrk_digest_rows(qrk_ctx* ctx, size_t n, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len,
                    uint8_t* out, void* stream) {
  if (!ctx) return fail("null context");
  if (n && (!a || !out || (b_len && !b))) return fail("null buffer");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  hipError_t e = digest_rows(n, a, a_len, b_len ? b : nullptr, b_len, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("digest_rows", e);
}

int qrk_hqc_supports(qrk_ctx* ctx, const char* alg, int kind, size_t n, const uint32_t* r, uint32_t* sup,
                     void* stream) {
  QRK_RESOLVE(ctx, alg);
  if (a->family != Family::HQC) return fail(std::string("not an HQC parameter set: ") + alg);
  if (kind != 0 && kind != 1) return fail("kind must be 0 (w) or 1 (w_r = w_e)");
  if (n && (!r || !sup)) return fail("null buffer");
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  hipError_t e = hqc_supports(*a, kind, n, r, sup, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("hqc_supports", e);
}

int qrk_hkdf_sha256_batch(qrk_ctx* ctx, size_t n, const uint8_t* ikm, size_t ikm_len, const uint8_t* salt,
                          size_t salt_len, const uint8_t* info, const uint64_t* info_off, size_t info_len,
                          uint8_t* okm, size_t okm_len, void* stream) {
  if (!ctx) return fail("null context");
  if (okm_len == 0 || okm_len > 255 * 32) return fail("HKDF-SHA256 output length must be 1..8160 bytes");
  if (salt_len && !salt) return fail("salt_len > 0 with a NULL salt");
  if (n && (!ikm || !okm || (!info && (info_off || info_len)))) return fail("null buffer");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  hipError_t e = hkdf_sha256(n, ikm, ikm_len, ikm_len, salt, salt_len, info, info_off, info_len, okm_len, okm,
                             okm_len, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("hkdf_sha256", e);
}

int qrk_handshake_batch(qrk_ctx* ctx, const char* alg, size_t n, const uint8_t* coins_kp_i,
                        const uint8_t* coins_kp_r, const uint8_t* coins_enc, const uint8_t* info,
                        const uint64_t* info_off, size_t info_len, size_t key_len, uint8_t* pk_i, uint8_t* pk_r,
                        uint8_t* ct, uint8_t* key_i, uint8_t* key_r, int32_t* agree, void* stream) {
  QRK_RESOLVE(ctx, alg);
  if (key_len == 0 || key_len > 255 * 32) return fail("key_len must be 1..8160 bytes");
  if (n == 0) return 0;
  if (!pk_i || !pk_r || !ct || !key_i || !key_r) return fail("null output buffer");
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  hipStream_t st = (hipStream_t)stream;
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  if (ctx_order(ctx, st)) return -1;
  LastUse last_use{ctx, st};
  // Ephemeral secrets of one chunk live in context scratch and are wiped afterwards
  // (the reference keeps them in Python objects: messaging.py:590-600, 809).
  const size_t chunk = chunk_for(ctx, *a);
  const size_t m0 = std::min(chunk, n);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t b_sk = al(m0 * a->sk), b_ss = al(m0 * a->ss);
  // ML-KEM batched chunks: the initiator's sampled matrix A_hat, kept from its KeyGen (:590) for its
  // Decaps (:1038) -- the same rho, so Decaps skips K^2 SampleNTT entries (27 of a handshake's ~174
  // ML-KEM-768 permutations).  Public data (a function of rho): outside the wiped range.
  const bool keep_a = a->family == Family::MLKEM && m0 > mlkem_small_max();
  const size_t b_mat = keep_a ? al(mlkem_matrix_bytes(*a, m0)) : 0;
  if (grow_device(ctx, (void**)&ctx->hs_scratch, &ctx->hs_scratch_bytes, 2 * b_sk + 2 * b_ss + b_mat, st)) return -1;
  uint8_t *sk_i = ctx->hs_scratch, *sk_r = sk_i + b_sk, *ss_i = sk_r + b_sk, *ss_r = ss_i + b_ss;
  uint64_t* mat_i = keep_a ? (uint64_t*)(ss_r + b_ss) : nullptr;
  struct NextReset {  // the hand-over fields never outlive one run_batch call
    qrk_ctx* c;
    ~NextReset() { c->xof_keep_next = nullptr, c->xof_given_next = nullptr; }
  } next_reset{ctx};
  // wipes the ephemeral sk / ss on every exit path, error returns included (runs before
  // last_use records the end of the call)
  struct Wipe {
    void* p;
    size_t bytes;
    hipStream_t st;
    ~Wipe() { (void)hipMemsetAsync(p, 0, bytes, st); }
  } wipe{ctx->hs_scratch, 2 * b_sk + 2 * b_ss, st};
  for (size_t off = 0; off < n; off += chunk) {
    const size_t m = std::min(chunk, n - off);
    auto co = [&](const uint8_t* c, size_t len) { return c ? c + off * len : nullptr; };
    // initiate_key_exchange: ephemeral KeyGen (messaging.py:590); A_hat kept for its Decaps
    const bool keep = keep_a && m > mlkem_small_max();
    ctx->xof_keep_next = keep ? mat_i : nullptr;
    const int rc_kg = run_batch(ctx, *a, Op::KEYPAIR, m, pk_i + off * a->pk, sk_i, co(coins_kp_i, a->kp_coins), nullptr,
                                nullptr, st);
    ctx->xof_keep_next = nullptr;
    if (rc_kg) return -1;
    // _handle_key_exchange_init: responder KeyGen (:809, pk sent back at :853) + Encaps (:830)
    if (run_batch(ctx, *a, Op::KEYPAIR, m, pk_r + off * a->pk, sk_r, co(coins_kp_r, a->kp_coins), nullptr, nullptr,
                  st))
      return -1;
    if (run_batch(ctx, *a, Op::ENCAPS, m, ct + off * a->ct, ss_r, pk_i + off * a->pk, co(coins_enc, a->enc_coins),
                  nullptr, st))
      return -1;
    hipError_t e = hkdf_sha256(m, ss_r, a->ss, a->ss, nullptr, 0, info, info_off ? info_off + off : nullptr,
                               info_len, key_len, key_r + off * key_len, key_len, st);  // :845
    if (e != hipSuccess) return hip_fail("hkdf_sha256", e);
    // _handle_key_exchange_response: Decaps (:1038) + HKDF (:1068)
    ctx->xof_given_next = keep ? mat_i : nullptr;
    const int rc_dec = run_batch(ctx, *a, Op::DECAPS, m, ss_i, nullptr, ct + off * a->ct, sk_i, nullptr, st);
    ctx->xof_given_next = nullptr;
    if (rc_dec) return -1;
    e = hkdf_sha256(m, ss_i, a->ss, a->ss, nullptr, 0, info, info_off ? info_off + off : nullptr, info_len,
                    key_len, key_i + off * key_len, key_len, st);
    if (e != hipSuccess) return hip_fail("hkdf_sha256", e);
    if (agree) {
      e = keys_equal(m, key_i + off * key_len, key_r + off * key_len, key_len, agree + off, st);
      if (e != hipSuccess) return hip_fail("keys_equal", e);
    }
  }
  return 0;
}

int qrk_base64_encode_batch(qrk_ctx* ctx, size_t n, const uint8_t* in, size_t in_len, uint8_t* out, void* stream) {
  if (!ctx) return fail("null context");
  if (n && in_len && (!in || !out)) return fail("null buffer");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  hipError_t e = base64_encode(n, in, in_len, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("base64_encode", e);
}

int qrk_base64_decode_batch(qrk_ctx* ctx, size_t n, const uint8_t* in, size_t out_len, uint8_t* out, int32_t* status,
                            void* stream) {
  if (!ctx) return fail("null context");
  if (n && out_len && (!in || !out)) return fail("null buffer");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard device_guard;
  if (device_guard.set(ctx->device)) return -1;
  TimerScope timer_scope(ctx->profiling ? &ctx->timer : nullptr);
  hipError_t e = hipSuccess;
  if (status && n) e = hipMemsetAsync(status, 0, n * sizeof(int32_t), (hipStream_t)stream);
  if (e == hipSuccess) e = base64_decode(n, in, out_len, out, status, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail("base64_decode", e);
}

const char* qrk_last_error(void) { return g_err.c_str(); }

int qrk_device_count(void) {
  int c = 0;
  return hipGetDeviceCount(&c) == hipSuccess ? c : 0;
}

}  // extern "C"
