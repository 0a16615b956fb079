// capi.hip -- host side of libssnt_tts_c: the reference's seven extern "C" symbols (host
// pointers, synchronous, abort on contract violation) and the device-pointer extensions.
//
// Reference symbols (ssnt_tts_c/src/lib.rs) take host arrays owned by the TF op for the call
// only. Each call here packs its inputs into one pinned staging buffer, does
// one H2D copy, launches the HIP kernel(s) and one D2H copy on the calling thread's own stream,
// then synchronises. Streams and scratch are thread_local: TF calls ops from several inter-op
// threads concurrently and the calls share nothing.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>

#include "ssnt_internal.h"

namespace ssnt {

int status_bits_to_code(int bits) {
  if (bits & kStatusNoCandidate) return SSNT_ERR_NO_CANDIDATE;
  if (bits & kStatusDurationMismatch) return SSNT_ERR_DURATION_MISMATCH;
  if (bits & kStatusBadLength) return SSNT_ERR_BAD_LENGTH;
  if (bits & kStatusBadIndex) return SSNT_ERR_BAD_INDEX;
  if (bits & (kStatusTimeout | kStatusRingTag)) return SSNT_ERR_INTERNAL;  // (tags: diag builds)
  return SSNT_OK;
}

namespace {

[[noreturn]] void fail(const char* fn, const char* msg) {
  // mirrors a Rust panic escaping an extern fn: the process aborts
  fprintf(stderr, "libssnt_tts_c: %s: %s\n", fn, msg);
  fflush(stderr);
  abort();
}

void check_ptr(const void* p, const char* fn, const char* name) {
  if (p == nullptr) {
    char buf[128];
    snprintf(buf, sizeof buf, "assertion failed: !%s.is_null()", name);
    fail(fn, buf);
  }
}

// Per-thread GPU context: stream, device scratch, pinned staging, status word.
struct HostCtx {
  int device = -1;
  hipStream_t stream = nullptr;
  char* d = nullptr;
  size_t dcap = 0;
  char* h = nullptr;
  size_t hcap = 0;
  char* hmap = nullptr;       // device address of the pinned staging buffer (zero-copy plans)
  unsigned* flag_h = nullptr;  // completion word in coherent pinned memory (host side) ...
  unsigned* flag_d = nullptr;  // ... and its device address
  unsigned seq = 0;            // last completion value requested
};
thread_local HostCtx g_ctx;

int ctx_ready(const char* fn, bool abort_on_error) {
  int dev = -1;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    if (abort_on_error) fail(fn, "no HIP device available (libssnt_tts_c has no CPU fallback)");
    return SSNT_ERR_HIP;
  }
  if (hipGetDevice(&dev) != hipSuccess) {
    if (abort_on_error) fail(fn, "hipGetDevice failed");
    return SSNT_ERR_HIP;
  }
  if (g_ctx.device != dev) {
    // a different device for this thread: release the old device's stream and buffers (HIP
    // frees device allocations and streams from any current device)
    if (g_ctx.stream) {
      (void)hipStreamSynchronize(g_ctx.stream);
      (void)hipStreamDestroy(g_ctx.stream);
    }
    if (g_ctx.d) (void)hipFree(g_ctx.d);
    if (g_ctx.h) (void)hipHostFree(g_ctx.h);
    if (g_ctx.flag_h) (void)hipHostFree(g_ctx.flag_h);
    g_ctx = HostCtx{};
    g_ctx.device = dev;
    if (hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking) != hipSuccess) {
      if (abort_on_error) fail(fn, "hipStreamCreate failed");
      return SSNT_ERR_HIP;
    }
    // the completion word of the per-step symbols: coherent (uncached) pinned memory, so a GPU
    // write of it is visible to the polling host thread without a cache flush
    void* fh = nullptr;
    void* fd = nullptr;
    if (hipHostMalloc(&fh, 4096, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
        hipHostGetDevicePointer(&fd, fh, 0) == hipSuccess && fd) {
      g_ctx.flag_h = static_cast<unsigned*>(fh);
      g_ctx.flag_d = static_cast<unsigned*>(fd);
      *g_ctx.flag_h = 0;
    } else if (fh) {
      (void)hipHostFree(fh);
    }
  }
  return SSNT_OK;
}

int ensure(size_t dbytes, size_t hbytes, const char* fn, bool abort_on_error) {
  if (dbytes > g_ctx.dcap) {
    if (g_ctx.d) {
      (void)hipStreamSynchronize(g_ctx.stream);
      (void)hipFree(g_ctx.d);
    }
    g_ctx.d = nullptr;
    g_ctx.dcap = 0;
    const size_t cap = dbytes + dbytes / 2 + 4096;
    if (hipMalloc(reinterpret_cast<void**>(&g_ctx.d), cap) != hipSuccess) {
      if (abort_on_error) fail(fn, "hipMalloc failed");
      return SSNT_ERR_HIP;
    }
    g_ctx.dcap = cap;
  }
  if (hbytes > g_ctx.hcap) {
    if (g_ctx.h) {
      (void)hipStreamSynchronize(g_ctx.stream);
      (void)hipHostFree(g_ctx.h);
    }
    g_ctx.h = nullptr;
    g_ctx.hmap = nullptr;
    g_ctx.hcap = 0;
    const size_t cap = hbytes + hbytes / 2 + 4096;
    // coherent (fine-grained) and mapped: zero-copy plans are read and written by the kernel in
    // place and the caller learns of completion from a flag word, not a stream synchronisation,
    // so the kernel's stores must bypass the GPU caches (a coarse-grained buffer is only
    // guaranteed coherent at synchronisation points)
    if (hipHostMalloc(reinterpret_cast<void**>(&g_ctx.h), cap,
                      hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      if (abort_on_error) fail(fn, "hipHostMalloc failed");
      return SSNT_ERR_HIP;
    }
    g_ctx.hcap = cap;
  }
  return SSNT_OK;
}

// Per-phase host clock of the per-step reference symbols (tools/bench_step_symbols.py
// --breakdown; diagnostics, off unless enabled): 0 entry -> context ready, 1 -> inputs staged,
// 2 -> kernel launched, 3 -> synchronised (outputs visible), 4 -> outputs scattered.
struct PhaseClock {
  bool on = false;
  int calls = 0;
  double acc[5] = {0, 0, 0, 0, 0};
  std::chrono::steady_clock::time_point last;
  void start() {
    if (on) last = std::chrono::steady_clock::now();
  }
  void mark(int k) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    acc[k] += std::chrono::duration<double, std::micro>(now - last).count();
    last = now;
    if (k == 4) ++calls;
  }
};
thread_local PhaseClock g_clk;

// How a per-step call (zero-copy plan) learns that its kernel is done: 0 hipStreamSynchronize;
// 1 hipStreamWriteValue32 of a sequence number into a coherent pinned word after the kernel,
// polled by the calling thread; 2 the same word written by a one-thread kernel launched after
// it. A poll that sees nothing for kFlagTimeoutMs falls back to hipStreamSynchronize (which
// then reports a failed kernel). Default measured per DESIGN.md 7.2 (tools/bench_step_symbols.py).
#ifdef SSNT_AB
std::atomic<int> g_sync_mode{2};  // A/B build: ssnt_set_host_sync
int sync_mode() { return g_sync_mode.load(std::memory_order_relaxed); }
#else
constexpr int sync_mode() { return 2; }
#endif
constexpr double kFlagTimeoutMs = 5000.0;

__global__ void k_flag(unsigned* f, unsigned v) {
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// enqueue the completion write behind the calling thread's kernels and spin until it lands;
// false: not seen (the caller synchronises)
bool wait_flag(int mode) {
  const unsigned seq = ++g_ctx.seq;
  if (mode == 1) {
    if (hipStreamWriteValue32(g_ctx.stream, g_ctx.flag_d, seq, 0) != hipSuccess) return false;
  } else {
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(1), 0, g_ctx.stream, g_ctx.flag_d, seq);
    if (hipGetLastError() != hipSuccess) return false;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned long n = 0;; ++n) {
    if (__atomic_load_n(g_ctx.flag_h, __ATOMIC_ACQUIRE) == seq) return true;
    if ((n & 1023) == 1023 &&
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > kFlagTimeoutMs)
      return false;
    __builtin_ia32_pause();
  }
}

// Host staging mode for the small per-step reference symbols (not ssnt_fwd_bwd, whose tensors
// are large): 0 = one H2D copy of inputs + zeroed status word, kernel, one D2H copy; 1 =
// zero-copy: the kernel reads its inputs from and writes its outputs to the pinned staging
// buffer over the bus (no copies; launch + synchronise only). Default measured per DESIGN.md
// (tools/bench_step_symbols.py); atomic, so concurrent callers never race on it.
#ifdef SSNT_AB
std::atomic<int> g_host_mode{1};  // A/B build: ssnt_set_host_staging
int host_mode() { return g_host_mode.load(std::memory_order_relaxed); }
#else
constexpr int host_mode() { return 1; }
#endif
constexpr size_t kZeroCopyMax = 1 << 20;  // plans up to this size may run zero-copy

// Staging plan: a list of host arrays laid out in one buffer: inputs, the status word, then the
// outputs, so a single H2D copy covers the inputs and the zeroed status word.
struct Slot {
  const void* src;  // host input (null for pure outputs)
  void* dst;        // host output (null for pure inputs)
  size_t bytes;
  size_t off;
};

struct Plan {
  std::vector<Slot> in, out;
  size_t status_off = 0, total = 0;
  bool zero_copy = false;
  char* dbase = nullptr;  // what the kernel addresses: device scratch, or the mapped staging buffer
  static size_t align(size_t x) { return (x + 255) & ~size_t(255); }
  int add_in(const void* src, size_t bytes) {
    in.push_back(Slot{src, nullptr, bytes, 0});
    return (int)in.size() - 1;
  }
  int add_out(void* dst, size_t bytes, const void* init = nullptr) {
    out.push_back(Slot{init, dst, bytes, 0});
    return (int)out.size() - 1;
  }
  void layout() {
    size_t o = 0;
    for (auto& s : in) { s.off = o; o += align(s.bytes); }
    status_off = o;
    o += 256;
    // outputs that need their previous contents (init) are uploaded too
    for (auto& s : out) { s.off = o; o += align(s.bytes); }
    total = o;
  }
  template <typename T> T* din(int i) const { return reinterpret_cast<T*>(dbase + in[i].off); }
  template <typename T> T* dout(int i) const { return reinterpret_cast<T*>(dbase + out[i].off); }
  int* dstatus() const { return reinterpret_cast<int*>(dbase + status_off); }
};

// Stage inputs (and output init contents) and a zeroed status word: one H2D copy, or none in
// zero-copy mode. `allow_zero_copy`: the per-step symbols only.
int stage_in(Plan& p, const char* fn, bool abort_on_error, size_t extra_device = 0,
             bool allow_zero_copy = true) {
  p.layout();
  p.zero_copy = allow_zero_copy && extra_device == 0 && p.total <= kZeroCopyMax &&
                host_mode() == 1;
  int rc = ensure(p.zero_copy ? 0 : Plan::align(p.total) + extra_device, p.total, fn,
                  abort_on_error);
  if (rc != SSNT_OK) return rc;
  if (p.zero_copy) {
    void* mapped = g_ctx.hmap;  // looked up once per staging allocation
    if (!mapped && (hipHostGetDevicePointer(&mapped, g_ctx.h, 0) != hipSuccess || mapped == nullptr)) {
      mapped = nullptr;
      p.zero_copy = false;  // not mappable here: fall back to the copies
      rc = ensure(Plan::align(p.total) + extra_device, p.total, fn, abort_on_error);
      if (rc != SSNT_OK) return rc;
    } else {
      g_ctx.hmap = static_cast<char*>(mapped);
      p.dbase = g_ctx.hmap;
    }
  }
  if (!p.zero_copy) p.dbase = g_ctx.d;
  for (auto& s : p.in) memcpy(g_ctx.h + s.off, s.src, s.bytes);
  memset(g_ctx.h + p.status_off, 0, sizeof(int));
  size_t up_end = p.status_off + sizeof(int);
  for (auto& s : p.out)
    if (s.src) {
      memcpy(g_ctx.h + s.off, s.src, s.bytes);
      up_end = s.off + s.bytes;
    }
  if (p.zero_copy) {
    g_clk.mark(1);
    return SSNT_OK;
  }
  const hipError_t e = hipMemcpyAsync(g_ctx.d, g_ctx.h, up_end, hipMemcpyHostToDevice, g_ctx.stream);
  g_clk.mark(1);
  if (e != hipSuccess) {
    if (abort_on_error) fail(fn, hipGetErrorString(e));
    return SSNT_ERR_HIP;
  }
  return SSNT_OK;
}

// Download status + outputs (one D2H copy, none in zero-copy mode), synchronise, scatter to the
// caller's arrays. Returns status code.
int stage_out(Plan& p, int launch_rc, const char* fn, bool abort_on_error) {
  g_clk.mark(2);
  if (launch_rc != SSNT_OK) {
    if (abort_on_error) fail(fn, ssnt_status_string(launch_rc));
    return launch_rc;
  }
  hipError_t e = hipSuccess;
  if (!p.zero_copy) {
    const size_t lo = p.status_off, hi = p.total;
    e = hipMemcpyAsync(g_ctx.h + lo, g_ctx.d + lo, hi - lo, hipMemcpyDeviceToHost, g_ctx.stream);
  }
  const int sm = sync_mode();
  if (e == hipSuccess && p.zero_copy && sm != 0 && g_ctx.flag_h && wait_flag(sm))
    ;  // completion seen through the flag word: the outputs are in the staging buffer
  else if (e == hipSuccess)
    e = hipStreamSynchronize(g_ctx.stream);
  if (e != hipSuccess) {
    if (abort_on_error) fail(fn, hipGetErrorString(e));
    return SSNT_ERR_HIP;
  }
  g_clk.mark(3);
  int bits = 0;
  memcpy(&bits, g_ctx.h + p.status_off, sizeof(int));
  const int rc = status_bits_to_code(bits);
  if (rc != SSNT_OK) {
    if (abort_on_error) {
      if (rc == SSNT_ERR_NO_CANDIDATE)
        fail(fn, "assertion failed: Beam search could not find a duration sequence with "
                 "compatible output length. Please increase duration class size and beam width.");
      if (rc == SSNT_ERR_DURATION_MISMATCH)
        fail(fn, "assertion failed: `(left == right)`: upsampled.len() != output_length");
      fail(fn, ssnt_status_string(rc));
    }
    return rc;
  }
  for (auto& s : p.out) memcpy(s.dst, g_ctx.h + s.off, s.bytes);
  g_clk.mark(4);
  return SSNT_OK;
}

__global__ void k_null() {}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace
}  // namespace ssnt

using namespace ssnt;

// the C ABI is the library's only exported surface (everything else builds -fvisibility=hidden)
#pragma GCC visibility push(default)
extern "C" {

const char* ssnt_status_string(int status) {
  switch (status) {
    case SSNT_OK: return "ok";
    case SSNT_ERR_INVALID_ARG: return "invalid argument";
    case SSNT_ERR_HIP: return "HIP runtime error";
    case SSNT_ERR_NO_CANDIDATE: return "v2 beam search found no candidate (src/v2.rs:292)";
    case SSNT_ERR_DURATION_MISMATCH: return "duration sum != output_length (src/v2_util.rs:58)";
    case SSNT_ERR_UNSUPPORTED: return "size not supported by the kernels";
    case SSNT_ERR_WORKSPACE: return "workspace missing or too small";
    case SSNT_ERR_BAD_LENGTH: return "length exceeds tensor extent";
    case SSNT_ERR_BAD_INDEX: return "beam branch index out of range";
    case SSNT_ERR_INTERNAL: return "internal: a bounded intra-kernel wait expired";
    default: return "unknown status";
  }
}

int ssnt_status_from_bits(int bits) { return status_bits_to_code(bits); }

int ssnt_version(char* buf, size_t len) {
  if (buf && len) snprintf(buf, len, "libssnt_tts_c mi355x gfx950 (HIP %d.%d)", HIP_VERSION_MAJOR, HIP_VERSION_MINOR);
  return SSNT_OK;
}

// ------------------------------- reference symbols -------------------------------------------

void ssnt_tts_beam_search_decode(const float* h, const float* log_prob_history,
                                 const bool* is_finished, const int* t, const int* u, int max_t,
                                 int beam_width, int* prediction, float* log_probs, int* next_t,
                                 int* next_u, bool* next_is_finished, int* beam_branch) {
  static const char* fn = "ssnt_tts_beam_search_decode";
  check_ptr(h, fn, "h"); check_ptr(log_prob_history, fn, "log_prob_history");
  check_ptr(is_finished, fn, "is_finished"); check_ptr(t, fn, "t"); check_ptr(u, fn, "u");
  check_ptr(prediction, fn, "prediction"); check_ptr(log_probs, fn, "log_probs");
  check_ptr(next_t, fn, "next_t"); check_ptr(next_u, fn, "next_u");
  check_ptr(next_is_finished, fn, "next_is_finished"); check_ptr(beam_branch, fn, "beam_branch");
  if (beam_width <= 0) fail(fn, "chunk size must be non-zero (beam_width <= 0)");
  g_clk.start();
  ctx_ready(fn, true);
  g_clk.mark(0);
  const size_t W = beam_width;
  Plan p;
  const int ih = p.add_in(h, W * 2 * 4), ihist = p.add_in(log_prob_history, W * 4),
            ifin = p.add_in(is_finished, W), it = p.add_in(t, W * 4), iu = p.add_in(u, W * 4);
  const int op = p.add_out(prediction, W * 4), ol = p.add_out(log_probs, W * 4),
            ot = p.add_out(next_t, W * 4), ou = p.add_out(next_u, W * 4),
            of = p.add_out(next_is_finished, W), ob = p.add_out(beam_branch, W * 4);
  stage_in(p, fn, true);
  StepArgs a{};
  a.variant = Variant::V1;
  a.B = 1; a.W = beam_width; a.Wmax = beam_width; a.C = 2;
  a.h = p.din<float>(ih); a.hist = p.din<float>(ihist); a.fin = p.din<bool>(ifin);
  a.t = p.din<int>(it); a.u = p.din<int>(iu);
  a.input_length = nullptr; a.scalar_input_length = max_t;
  a.prediction = p.dout<int>(op); a.log_prob = p.dout<float>(ol); a.next_t = p.dout<int>(ot);
  a.next_u = p.dout<int>(ou); a.next_fin = p.dout<bool>(of); a.beam_branch = p.dout<int>(ob);
  a.status = p.dstatus();
  stage_out(p, launch_decode_step(a, g_ctx.stream), fn, true);
}

void ssnt_extract_best_beam_branch(int best_final_branch, const int* beam_branch,
                                   const int* t_history, int beam_width, int max_u,
                                   int* best_beam_branch, int* best_t_history) {
  static const char* fn = "ssnt_extract_best_beam_branch";
  check_ptr(beam_branch, fn, "beam_branch"); check_ptr(t_history, fn, "t_history");
  check_ptr(best_beam_branch, fn, "best_beam_branch");
  check_ptr(best_t_history, fn, "best_t_history");
  if (beam_width <= 0 || max_u < 0) fail(fn, "chunk size must be non-zero (beam_width <= 0)");
  if (max_u == 0) return;
  ctx_ready(fn, true);
  const size_t n = (size_t)max_u * beam_width;
  Plan p;
  const int ifb = p.add_in(&best_final_branch, 4), ib = p.add_in(beam_branch, n * 4),
            ith = p.add_in(t_history, n * 4);
  const int ob = p.add_out(best_beam_branch, (size_t)max_u * 4),
            ot = p.add_out(best_t_history, (size_t)max_u * 4);
  stage_in(p, fn, true);
  const int rc = launch_extract_best(1, beam_width, max_u, p.din<int>(ifb), p.din<int>(ib),
                                     p.din<int>(ith), p.dout<int>(ob), p.dout<int>(ot),
                                     p.dstatus(), g_ctx.stream);
  stage_out(p, rc, fn, true);
}

void ssnt_tts_v2_beam_search_decode(const float* h, const float* log_prob_history,
                                    const bool* is_finished, const int* total_duration,
                                    const int* duration_table, const int* t, const int* u,
                                    const int* input_length, const int* output_length,
                                    int batch_size, int beam_width, int duration_class_size,
                                    int zero_duration_id, bool allow_skip, bool test_mode,
                                    int* prediction, float* log_probs, int* next_t, int* next_u,
                                    bool* next_is_finished, int* next_total_duration,
                                    int* beam_branch) {
  static const char* fn = "ssnt_tts_v2_beam_search_decode";
  check_ptr(h, fn, "h"); check_ptr(log_prob_history, fn, "log_prob_history");
  check_ptr(is_finished, fn, "is_finished"); check_ptr(total_duration, fn, "total_duration");
  check_ptr(duration_table, fn, "duration_table"); check_ptr(t, fn, "t"); check_ptr(u, fn, "u");
  check_ptr(input_length, fn, "input_length"); check_ptr(output_length, fn, "output_length");
  check_ptr(prediction, fn, "prediction"); check_ptr(log_probs, fn, "log_probs");
  check_ptr(next_t, fn, "next_t"); check_ptr(next_u, fn, "next_u");
  check_ptr(next_is_finished, fn, "next_is_finished");
  check_ptr(next_total_duration, fn, "next_total_duration");
  check_ptr(beam_branch, fn, "beam_branch");
  if (batch_size < 0 || beam_width <= 0 || duration_class_size <= 0)
    fail(fn, "chunk size must be non-zero (beam_width / duration_class_size <= 0)");
  if (batch_size == 0) return;
  ctx_ready(fn, true);
  const size_t BW = (size_t)batch_size * beam_width, D = duration_class_size;
  Plan p;
  const int ih = p.add_in(h, BW * D * 4), ihist = p.add_in(log_prob_history, BW * 4),
            ifin = p.add_in(is_finished, BW), itot = p.add_in(total_duration, BW * 4),
            itab = p.add_in(duration_table, D * 4), it = p.add_in(t, BW * 4),
            iu = p.add_in(u, BW * 4), iil = p.add_in(input_length, (size_t)batch_size * 4),
            iol = p.add_in(output_length, (size_t)batch_size * 4);
  const int op = p.add_out(prediction, BW * 4), ol = p.add_out(log_probs, BW * 4),
            ot = p.add_out(next_t, BW * 4), ou = p.add_out(next_u, BW * 4),
            of = p.add_out(next_is_finished, BW), otd = p.add_out(next_total_duration, BW * 4),
            ob = p.add_out(beam_branch, BW * 4);
  stage_in(p, fn, true);
  StepArgs a{};
  a.variant = Variant::V2;
  a.B = batch_size; a.W = beam_width; a.Wmax = beam_width; a.C = duration_class_size;
  a.h = p.din<float>(ih); a.hist = p.din<float>(ihist); a.fin = p.din<bool>(ifin);
  a.total = p.din<int>(itot); a.table = p.din<int>(itab);
  a.t = p.din<int>(it); a.u = p.din<int>(iu);
  a.input_length = p.din<int>(iil); a.output_length = p.din<int>(iol);
  a.special_id = zero_duration_id; a.allow_skip = allow_skip; a.test_mode = test_mode;
  a.prediction = p.dout<int>(op); a.log_prob = p.dout<float>(ol); a.next_t = p.dout<int>(ot);
  a.next_u = p.dout<int>(ou); a.next_fin = p.dout<bool>(of); a.next_total = p.dout<int>(otd);
  a.beam_branch = p.dout<int>(ob);
  a.status = p.dstatus();
  stage_out(p, launch_decode_step(a, g_ctx.stream), fn, true);
}

void ssnt_order_beam_branch(const int* final_branch, const int* beam_branch, int batch_size,
                            int beam_width, int max_t, int* ordered_beam_branch) {
  static const char* fn = "ssnt_order_beam_branch";
  check_ptr(final_branch, fn, "final_branch"); check_ptr(beam_branch, fn, "beam_branch");
  check_ptr(ordered_beam_branch, fn, "ordered_beam_branch");
  if (batch_size < 0 || beam_width <= 0 || max_t <= 0)
    fail(fn, "chunk size must be non-zero (beam_width / max_t <= 0)");
  if (batch_size == 0) return;
  ctx_ready(fn, true);
  const size_t BW = (size_t)batch_size * beam_width;
  Plan p;
  const int ifb = p.add_in(final_branch, BW * 4), ib = p.add_in(beam_branch, BW * max_t * 4);
  const int oo = p.add_out(ordered_beam_branch, BW * max_t * 4);
  stage_in(p, fn, true);
  const int rc = launch_order_beam_branch(batch_size, beam_width, max_t, p.din<int>(ifb),
                                          p.din<int>(ib), p.dout<int>(oo), p.dstatus(),
                                          g_ctx.stream);
  stage_out(p, rc, fn, true);
}

void ssnt_upsample_source_indexes(const int* duration, const int* output_length, int batch_size,
                                  int beam_width, int max_t, int max_u,
                                  int* upsampled_source_indexes) {
  static const char* fn = "ssnt_upsample_source_indexes";
  check_ptr(duration, fn, "duration"); check_ptr(output_length, fn, "output_length");
  check_ptr(upsampled_source_indexes, fn, "upsampled_source_indexes");
  if (batch_size < 0 || beam_width <= 0 || max_t <= 0 || max_u <= 0)
    fail(fn, "chunk size must be non-zero (beam_width / max_t / max_u <= 0)");
  if (batch_size == 0) return;
  ctx_ready(fn, true);
  const size_t BW = (size_t)batch_size * beam_width;
  Plan p;
  const int id = p.add_in(duration, BW * max_t * 4), il = p.add_in(output_length, BW * 4);
  // rows are written only up to output_length: upload the caller's prefill (the TF op fills
  // out_of_range_source_index, upsample_source_indexes_op.cc:75) so it survives the download
  const int oo = p.add_out(upsampled_source_indexes, BW * max_u * 4, upsampled_source_indexes);
  stage_in(p, fn, true);
  const int rc = launch_upsample(batch_size, beam_width, max_t, max_u, p.din<int>(id),
                                 p.din<int>(il), p.dout<int>(oo), p.dstatus(), g_ctx.stream);
  stage_out(p, rc, fn, true);
}

void tone_latent_beam_search_decode(const float* h, const float* log_prob_history,
                                    const bool* is_finished, const int* t, const int* u,
                                    const int* input_length, int batch_size, int beam_width,
                                    int tone_class_size, int empty_tone_id, int* prediction,
                                    float* log_probs, int* next_t, int* next_u,
                                    bool* next_is_finished, int* beam_branch) {
  static const char* fn = "tone_latent_beam_search_decode";
  check_ptr(h, fn, "h"); check_ptr(log_prob_history, fn, "log_prob_history");
  check_ptr(is_finished, fn, "is_finished"); check_ptr(t, fn, "t"); check_ptr(u, fn, "u");
  check_ptr(input_length, fn, "input_length"); check_ptr(prediction, fn, "prediction");
  check_ptr(log_probs, fn, "log_probs"); check_ptr(next_t, fn, "next_t");
  check_ptr(next_u, fn, "next_u"); check_ptr(next_is_finished, fn, "next_is_finished");
  check_ptr(beam_branch, fn, "beam_branch");
  if (batch_size < 0 || beam_width <= 0 || tone_class_size <= 0)
    fail(fn, "chunk size must be non-zero (beam_width / tone_class_size <= 0)");
  if (batch_size == 0) return;
  ctx_ready(fn, true);
  const size_t BW = (size_t)batch_size * beam_width, C = tone_class_size;
  Plan p;
  const int ih = p.add_in(h, BW * C * 4), ihist = p.add_in(log_prob_history, BW * 4),
            ifin = p.add_in(is_finished, BW), it = p.add_in(t, BW * 4), iu = p.add_in(u, BW * 4),
            iil = p.add_in(input_length, (size_t)batch_size * 4);
  const int op = p.add_out(prediction, BW * 4), ol = p.add_out(log_probs, BW * 4),
            ot = p.add_out(next_t, BW * 4), ou = p.add_out(next_u, BW * 4),
            of = p.add_out(next_is_finished, BW), ob = p.add_out(beam_branch, BW * 4);
  stage_in(p, fn, true);
  StepArgs a{};
  a.variant = Variant::Tone;
  a.B = batch_size; a.W = beam_width; a.Wmax = beam_width; a.C = tone_class_size;
  a.h = p.din<float>(ih); a.hist = p.din<float>(ihist); a.fin = p.din<bool>(ifin);
  a.t = p.din<int>(it); a.u = p.din<int>(iu); a.input_length = p.din<int>(iil);
  a.special_id = empty_tone_id;
  a.prediction = p.dout<int>(op); a.log_prob = p.dout<float>(ol); a.next_t = p.dout<int>(ot);
  a.next_u = p.dout<int>(ou); a.next_fin = p.dout<bool>(of); a.beam_branch = p.dout<int>(ob);
  a.status = p.dstatus();
  stage_out(p, launch_decode_step(a, g_ctx.stream), fn, true);
}

void tone_latent_levenshtein_edit_distance(const int* a, const int* b, const int* a_lengths,
                                           const int* b_lengths, int batch_size, int max_length,
                                           int* distance) {
  static const char* fn = "tone_latent_levenshtein_edit_distance";
  check_ptr(a, fn, "a"); check_ptr(b, fn, "b"); check_ptr(a_lengths, fn, "a_lengths");
  check_ptr(b_lengths, fn, "b_lengths"); check_ptr(distance, fn, "distance");
  if (batch_size < 0 || max_length < 0) fail(fn, "invalid batch_size / max_length");
  for (int i = 0; i < batch_size; ++i)  // `&a[..a_length]` slice bounds (src/edit_distance.rs:17-18)
    if (a_lengths[i] < 0 || a_lengths[i] > max_length || b_lengths[i] < 0 || b_lengths[i] > max_length)
      fail(fn, "range end index out of range for slice (length > max_length)");
  if (batch_size == 0) return;
  if (max_length == 0) {
    for (int i = 0; i < batch_size; ++i) distance[i] = 0;
    return;
  }
  ctx_ready(fn, true);
  const size_t n = (size_t)batch_size * max_length;
  Plan p;
  const int ia = p.add_in(a, n * 4), ib = p.add_in(b, n * 4),
            ial = p.add_in(a_lengths, (size_t)batch_size * 4),
            ibl = p.add_in(b_lengths, (size_t)batch_size * 4);
  const int od = p.add_out(distance, (size_t)batch_size * 4);
  stage_in(p, fn, true);
  const int rc = launch_levenshtein(batch_size, max_length, p.din<int>(ia), p.din<int>(ib),
                                    p.din<int>(ial), p.din<int>(ibl), p.dout<int>(od),
                                    g_ctx.stream);
  stage_out(p, rc, fn, true);
}

// ------------------------------- extensions ---------------------------------------------------

int ssnt_fwd_bwd_last_kernel(char* buf, size_t len) {
  const char* d = last_fwd_bwd_dispatch();
  if (buf && len) snprintf(buf, len, "%s", d);
  return (int)strlen(d);
}

// ---- A/B build only (-DSSNT_AB, lib/ab/libssnt_tts_c_ab.so; include/ssnt_tts_c_ab.h): the
// process-wide kernel / staging / sync knobs and the diagnostic reads. The product library
// exports none of them (tests/test_capi_exports.py).
#ifdef SSNT_AB
int ssnt_fwd_bwd_set_variant(int variant) { return set_fwd_bwd_variant(variant); }

// host staging of the per-step reference symbols (tools/bench_step_symbols.py): 0 = copies,
// 1 = zero-copy. Returns the previous mode.
int ssnt_set_host_staging(int mode) {
  if (mode != 0 && mode != 1) return -1;
  return g_host_mode.exchange(mode);
}

// how the per-step reference symbols wait for their kernel (g_sync_mode). Returns the previous
// mode.
int ssnt_set_host_sync(int mode) {
  if (mode < 0 || mode > 2) return -1;
  return g_sync_mode.exchange(mode);
}

// the fused decodes' step ordering: -1 default, 0 full rank, 1 selection
int ssnt_fused_decode_select(int mode) { return set_fused_decode_select(mode); }
// waves of the tone fused decode's rank (1, 2, 4; -1 the product's choice)
int ssnt_fused_decode_tone_waves(int n) { return set_fused_decode_tone_waves(n); }

// the long-row kernel's lane width
int ssnt_fwd_bwd_wide_lanes(int k) { return set_fwd_bwd_wide_lanes(k); }
// the long-row kernel's workgroup split (-1 auto, 0 one workgroup per direction, 1 two
// whenever a direction has 2+ segments)
int ssnt_fwd_bwd_wide_split(int mode) { return set_fwd_bwd_wide_split(mode); }
// the streaming kernel's ring depth (16 / 32 slots, rows in the workspace; 0 default)
int ssnt_fwd_bwd_stream_ring(int r) { return set_stream_ring(r); }

// Per-step symbol latency breakdown (tools/bench_step_symbols.py).
// enable = 1 resets and starts the calling thread's phase clock; 0 stops it and writes the mean
// microseconds of its 5 phases (PhaseClock) to out[0..4]; returns the number of calls timed.
int ssnt_diag_step_clock(int enable, double* out) {
  if (enable) {
    g_clk = PhaseClock{};
    g_clk.on = true;
    return 0;
  }
  g_clk.on = false;
  for (int k = 0; k < 5; ++k) out[k] = g_clk.calls ? g_clk.acc[k] / g_clk.calls : 0.0;
  return g_clk.calls;
}
// The floor under a per-step call: an empty kernel launched on the calling thread's stream, then
// hipStreamSynchronize, `reps` times: out[0] mean launch us, out[1] mean synchronise us.
int ssnt_diag_null_launch(int reps, double* out) {
  if (ctx_ready("ssnt_diag_null_launch", false) != SSNT_OK) return -1;
  double l = 0, sy = 0;
  for (int i = 0; i < reps; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_null, dim3(1), dim3(64), 0, g_ctx.stream);
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(g_ctx.stream);
    const auto t2 = std::chrono::steady_clock::now();
    l += std::chrono::duration<double, std::micro>(t1 - t0).count();
    sy += std::chrono::duration<double, std::micro>(t2 - t1).count();
  }
  out[0] = reps ? l / reps : 0;
  out[1] = reps ? sy / reps : 0;
  return reps;
}

// in-kernel stamps of the diagnostic builds (make lib-diag / lib-exp; -1 otherwise)
int ssnt_diag_read(void* host, size_t bytes) { return diag_read(host, bytes); }
int ssnt_diag_decode_read(void* host, size_t bytes) { return diag_decode_read(host, bytes); }


#endif  // SSNT_AB

size_t ssnt_fwd_bwd_sum_state_size(int batch) { return batch > 0 ? fwd_bwd_sum_state_bytes(batch) : 0; }

size_t ssnt_fwd_bwd_workspace_size(int batch, int max_steps, int max_pos) {
  if (batch <= 0 || max_steps <= 0 || max_pos <= 0) return 0;
  return fwd_bwd_workspace_bytes(batch, max_steps, max_pos);
}

int ssnt_fwd_bwd_device(const float* log_trans, const float* log_obs, const int* step_len,
                        const int* pos_len, int batch, int max_steps, int max_pos, int flags,
                        float* loss, float* grad_trans, float* grad_obs, float* log_alpha,
                        float* log_beta, void* workspace, size_t workspace_bytes, int* status,
                        void* stream) {
  FwdBwdArgs a{};
  a.log_trans = log_trans; a.log_obs = log_obs; a.step_len = step_len; a.pos_len = pos_len;
  a.B = batch; a.T = max_steps; a.U = max_pos; a.flags = flags;
  a.loss = loss; a.grad = grad_trans; a.grad_obs = grad_obs;
  a.log_alpha = log_alpha; a.log_beta = log_beta;
  a.workspace = workspace; a.workspace_bytes = workspace_bytes; a.status = status;
  return launch_fwd_bwd(a, as_stream(stream));
}

size_t ssnt_fwd_bwd_debug64_workspace_size(int batch, int max_steps, int max_pos) {
  if (batch <= 0 || max_steps <= 0 || max_pos <= 0) return 0;
  return fwd_bwd_debug64_workspace_bytes(batch, max_steps, max_pos);
}

int ssnt_fwd_bwd_debug64_device(const float* log_trans, const float* log_obs, const int* step_len,
                                const int* pos_len, int batch, int max_steps, int max_pos,
                                int flags, double* loss, float* grad_trans, float* grad_obs,
                                double* log_alpha, double* log_beta, void* workspace,
                                size_t workspace_bytes, int* status, void* stream) {
  FwdBwdArgs a{};
  a.log_trans = log_trans; a.log_obs = log_obs; a.step_len = step_len; a.pos_len = pos_len;
  a.B = batch; a.T = max_steps; a.U = max_pos; a.flags = flags;
  a.grad = grad_trans; a.grad_obs = grad_obs;
  a.workspace = workspace; a.workspace_bytes = workspace_bytes; a.status = status;
  if (!log_trans || !step_len || !pos_len) return SSNT_ERR_INVALID_ARG;
  if (grad_obs && !log_obs) return SSNT_ERR_INVALID_ARG;
  return launch_fwd_bwd_debug64(a, loss, log_alpha, log_beta, as_stream(stream));
}

int ssnt_fwd_bwd_sum_device(const float* log_trans, const float* log_obs, const int* step_len,
                            const int* pos_len, int batch, int max_steps, int max_pos, int flags,
                            float* loss, float* grad_trans, float* grad_obs, float* log_alpha,
                            float* log_beta, void* workspace, size_t workspace_bytes, int* status,
                            float* loss_sum, void* sum_state, void* stream) {
  if (!loss_sum) return SSNT_ERR_INVALID_ARG;
  FwdBwdArgs a{};
  a.log_trans = log_trans; a.log_obs = log_obs; a.step_len = step_len; a.pos_len = pos_len;
  a.B = batch; a.T = max_steps; a.U = max_pos; a.flags = flags;
  a.loss = loss; a.grad = grad_trans; a.grad_obs = grad_obs;
  a.log_alpha = log_alpha; a.log_beta = log_beta;
  a.workspace = workspace; a.workspace_bytes = workspace_bytes; a.status = status;
  a.loss_sum = loss_sum; a.sum_state = sum_state;
  return launch_fwd_bwd(a, as_stream(stream));
}

size_t ssnt_v2_fwd_bwd_workspace_size(int batch, int max_steps, int max_total, bool test_mode) {
  return v2_fwd_bwd_workspace_bytes(batch, max_steps, max_total, test_mode);
}

int ssnt_v2_fwd_bwd_device(const float* logits, const int* duration_table, const int* input_length,
                           const int* output_length, int batch, int max_steps,
                           int duration_class_size, int max_total, int zero_duration_id,
                           bool allow_skip, bool test_mode, int flags, float* loss, float* grad,
                           float* log_alpha, float* log_beta, void* workspace,
                           size_t workspace_bytes, int* status, void* stream) {
  if (max_total < 0 || max_total > (1 << 24)) return SSNT_ERR_INVALID_ARG;
  V2FwdBwdArgs a{};
  a.logits = logits; a.table = duration_table; a.input_length = input_length;
  a.output_length = output_length; a.B = batch; a.Imax = max_steps; a.D = duration_class_size;
  a.X = max_total + 1; a.zid = zero_duration_id; a.allow_skip = allow_skip;
  a.test_mode = test_mode; a.flags = flags; a.loss = loss; a.grad = grad;
  a.log_alpha = log_alpha; a.log_beta = log_beta; a.workspace = workspace;
  a.workspace_bytes = workspace_bytes; a.status = status;
  return launch_v2_fwd_bwd(a, as_stream(stream));
}

int ssnt_fwd_bwd(const float* log_trans, const float* log_obs, const int* step_len,
                 const int* pos_len, int batch, int max_steps, int max_pos, int flags,
                 float* loss, float* grad_trans, float* grad_obs, float* log_alpha,
                 float* log_beta) {
  static const char* fn = "ssnt_fwd_bwd";
  if (!log_trans || !step_len || !pos_len || !loss || batch < 0 || max_steps <= 0 || max_pos <= 0)
    return SSNT_ERR_INVALID_ARG;
  if (grad_obs && !log_obs) return SSNT_ERR_INVALID_ARG;
  if (batch == 0) return SSNT_OK;
  int rc = ctx_ready(fn, false);
  if (rc != SSNT_OK) return rc;
  const size_t cells = (size_t)batch * max_steps * max_pos;
  const size_t ws = fwd_bwd_workspace_bytes(batch, max_steps, max_pos);
  Plan p;
  const int ilt = p.add_in(log_trans, cells * 8), isl = p.add_in(step_len, (size_t)batch * 4),
            ipl = p.add_in(pos_len, (size_t)batch * 4);
  const int ilo = log_obs ? p.add_in(log_obs, cells * 4) : -1;
  const int ol = p.add_out(loss, (size_t)batch * 4);
  const int og = grad_trans ? p.add_out(grad_trans, cells * 8) : -1;
  const int ogo = grad_obs ? p.add_out(grad_obs, cells * 4) : -1;
  const int ola = log_alpha ? p.add_out(log_alpha, cells * 4) : -1;
  const int olb = log_beta ? p.add_out(log_beta, cells * 4) : -1;
  rc = stage_in(p, fn, false, ws, false);  // device-only workspace reserved after the plan
  if (rc != SSNT_OK) return rc;
  const size_t ws_off = Plan::align(p.total);
  FwdBwdArgs a{};
  a.log_trans = p.din<float>(ilt); a.log_obs = log_obs ? p.din<float>(ilo) : nullptr;
  a.step_len = p.din<int>(isl); a.pos_len = p.din<int>(ipl);
  a.B = batch; a.T = max_steps; a.U = max_pos; a.flags = flags;
  a.loss = p.dout<float>(ol);
  a.grad = og >= 0 ? p.dout<float>(og) : nullptr;
  a.grad_obs = ogo >= 0 ? p.dout<float>(ogo) : nullptr;
  a.log_alpha = ola >= 0 ? p.dout<float>(ola) : nullptr;
  a.log_beta = olb >= 0 ? p.dout<float>(olb) : nullptr;
  a.workspace = ws ? g_ctx.d + ws_off : nullptr;
  a.workspace_bytes = ws;
  a.status = p.dstatus();
  return stage_out(p, launch_fwd_bwd(a, g_ctx.stream), fn, false);
}

int ssnt_beam_search_decode_device(const float* h, const float* log_prob_history,
                                   const bool* is_finished, const int* t, const int* u,
                                   const int* input_length, int batch_size, int beam_width,
                                   int* prediction, float* log_probs, int* next_t, int* next_u,
                                   bool* next_is_finished, int* beam_branch, int* status,
                                   void* stream) {
  if (!h || !log_prob_history || !is_finished || !t || !u || !input_length || !prediction ||
      !log_probs || !next_t || !next_u || !next_is_finished || !beam_branch)
    return SSNT_ERR_INVALID_ARG;
  StepArgs a{};
  a.variant = Variant::V1;
  a.B = batch_size; a.W = beam_width; a.Wmax = beam_width; a.C = 2;
  a.h = h; a.hist = log_prob_history; a.fin = is_finished; a.t = t; a.u = u;
  a.input_length = input_length;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.beam_branch = beam_branch; a.status = status;
  return launch_decode_step(a, as_stream(stream));
}

int ssnt_v2_beam_search_decode_device(const float* h, const float* log_prob_history,
                                      const bool* is_finished, const int* total_duration,
                                      const int* duration_table, const int* t, const int* u,
                                      const int* input_length, const int* output_length,
                                      int batch_size, int beam_width, int duration_class_size,
                                      int zero_duration_id, bool allow_skip, bool test_mode,
                                      int* prediction, float* log_probs, int* next_t,
                                      int* next_u, bool* next_is_finished,
                                      int* next_total_duration, int* beam_branch, int* status,
                                      void* stream) {
  if (!h || !log_prob_history || !is_finished || !total_duration || !duration_table || !t || !u ||
      !input_length || !output_length || !prediction || !log_probs || !next_t || !next_u ||
      !next_is_finished || !next_total_duration || !beam_branch)
    return SSNT_ERR_INVALID_ARG;
  StepArgs a{};
  a.variant = Variant::V2;
  a.B = batch_size; a.W = beam_width; a.Wmax = beam_width; a.C = duration_class_size;
  a.h = h; a.hist = log_prob_history; a.fin = is_finished; a.total = total_duration;
  a.table = duration_table; a.t = t; a.u = u;
  a.input_length = input_length; a.output_length = output_length;
  a.special_id = zero_duration_id; a.allow_skip = allow_skip; a.test_mode = test_mode;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.next_total = next_total_duration;
  a.beam_branch = beam_branch; a.status = status;
  return launch_decode_step(a, as_stream(stream));
}

int ssnt_tone_latent_beam_search_decode_device(const float* h, const float* log_prob_history,
                                               const bool* is_finished, const int* t,
                                               const int* u, const int* input_length,
                                               int batch_size, int beam_width,
                                               int tone_class_size, int empty_tone_id,
                                               int* prediction, float* log_probs, int* next_t,
                                               int* next_u, bool* next_is_finished,
                                               int* beam_branch, int* status, void* stream) {
  if (!h || !log_prob_history || !is_finished || !t || !u || !input_length || !prediction ||
      !log_probs || !next_t || !next_u || !next_is_finished || !beam_branch)
    return SSNT_ERR_INVALID_ARG;
  StepArgs a{};
  a.variant = Variant::Tone;
  a.B = batch_size; a.W = beam_width; a.Wmax = beam_width; a.C = tone_class_size;
  a.h = h; a.hist = log_prob_history; a.fin = is_finished; a.t = t; a.u = u;
  a.input_length = input_length; a.special_id = empty_tone_id;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.beam_branch = beam_branch; a.status = status;
  return launch_decode_step(a, as_stream(stream));
}

int ssnt_lattice_beam_search_decode_device(const float* lattice, const int* input_length,
                                           int batch_size, int max_steps, int max_pos,
                                           int beam_width, int* prediction, float* log_probs,
                                           int* next_t, int* next_u, bool* next_is_finished,
                                           int* beam_branch, int* best_beam_branch,
                                           int* best_t_history, int* status, void* stream) {
  if (!lattice || !input_length || !prediction || !log_probs || !next_t || !next_u ||
      !next_is_finished || !beam_branch || !best_beam_branch || !best_t_history)
    return SSNT_ERR_INVALID_ARG;
  FusedDecodeArgs a{};
  a.variant = Variant::V1;
  a.B = batch_size; a.T = max_steps; a.U = max_pos; a.W = beam_width; a.C = 2;
  a.src = lattice; a.input_length = input_length;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.beam_branch = beam_branch;
  a.best_beam_branch = best_beam_branch; a.best_t_history = best_t_history; a.status = status;
  return launch_fused_decode(a, as_stream(stream));
}

int ssnt_v2_lattice_beam_search_decode_device(
    const float* logits, const int* duration_table, const int* input_length,
    const int* output_length, int batch_size, int max_steps, int beam_width,
    int duration_class_size, int zero_duration_id, bool allow_skip, bool test_mode,
    int* prediction, float* log_probs, int* next_t, int* next_u, bool* next_is_finished,
    int* next_total_duration, int* beam_branch, int* ordered_beam_branch, int* path_prediction,
    int* duration, int* status, void* stream) {
  if (!logits || !duration_table || !input_length || !output_length || !prediction ||
      !log_probs || !next_t || !next_u || !next_is_finished || !next_total_duration ||
      !beam_branch || duration_class_size <= 0)
    return SSNT_ERR_INVALID_ARG;
  FusedDecodeArgs a{};
  a.variant = Variant::V2;
  a.B = batch_size; a.T = max_steps; a.W = beam_width; a.C = duration_class_size;
  a.src = logits; a.table = duration_table;
  a.input_length = input_length; a.output_length = output_length;
  a.special_id = zero_duration_id; a.allow_skip = allow_skip; a.test_mode = test_mode;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.next_total = next_total_duration; a.beam_branch = beam_branch;
  a.ordered = ordered_beam_branch; a.path_pred = path_prediction; a.duration = duration;
  a.status = status;
  return launch_fused_decode(a, as_stream(stream));
}

int ssnt_tone_latent_lattice_beam_search_decode_device(
    const float* logits, const int* input_length, int batch_size, int max_steps, int beam_width,
    int tone_class_size, int empty_tone_id, int* prediction, float* log_probs, int* next_t,
    int* next_u, bool* next_is_finished, int* beam_branch, int* ordered_beam_branch,
    int* path_prediction, int* status, void* stream) {
  if (!logits || !input_length || !prediction || !log_probs || !next_t || !next_u ||
      !next_is_finished || !beam_branch || tone_class_size <= 0)
    return SSNT_ERR_INVALID_ARG;
  FusedDecodeArgs a{};
  a.variant = Variant::Tone;
  a.B = batch_size; a.T = max_steps; a.W = beam_width; a.C = tone_class_size;
  a.src = logits; a.input_length = input_length; a.special_id = empty_tone_id;
  a.prediction = prediction; a.log_prob = log_probs; a.next_t = next_t; a.next_u = next_u;
  a.next_fin = next_is_finished; a.beam_branch = beam_branch;
  a.ordered = ordered_beam_branch; a.path_pred = path_prediction;
  a.status = status;
  return launch_fused_decode(a, as_stream(stream));
}

int ssnt_extract_best_beam_branch_device(const int* best_final_branch, const int* beam_branch,
                                         const int* t_history, int batch_size, int beam_width,
                                         int max_u, int* best_beam_branch, int* best_t_history,
                                         int* status, void* stream) {
  if (!beam_branch || !t_history || !best_beam_branch || !best_t_history)
    return SSNT_ERR_INVALID_ARG;
  return launch_extract_best(batch_size, beam_width, max_u, best_final_branch, beam_branch,
                             t_history, best_beam_branch, best_t_history, status,
                             as_stream(stream));
}

int ssnt_order_beam_branch_device(const int* final_branch, const int* beam_branch,
                                  int batch_size, int beam_width, int max_t,
                                  int* ordered_beam_branch, int* status, void* stream) {
  if (!final_branch || !beam_branch || !ordered_beam_branch) return SSNT_ERR_INVALID_ARG;
  return launch_order_beam_branch(batch_size, beam_width, max_t, final_branch, beam_branch,
                                  ordered_beam_branch, status, as_stream(stream));
}

int ssnt_upsample_source_indexes_device(const int* duration, const int* output_length,
                                        int batch_size, int beam_width, int max_t, int max_u,
                                        int* upsampled_source_indexes, int* status,
                                        void* stream) {
  if (!duration || !output_length || !upsampled_source_indexes) return SSNT_ERR_INVALID_ARG;
  return launch_upsample(batch_size, beam_width, max_t, max_u, duration, output_length,
                         upsampled_source_indexes, status, as_stream(stream));
}

int ssnt_levenshtein_edit_distance_device(const int* a, const int* b, const int* a_lengths,
                                          const int* b_lengths, int batch_size, int max_length,
                                          int* distance, void* stream) {
  if (!a || !b || !a_lengths || !b_lengths || !distance) return SSNT_ERR_INVALID_ARG;
  return launch_levenshtein(batch_size, max_length, a, b, a_lengths, b_lengths, distance,
                            as_stream(stream));
}

}  // extern "C"
#pragma GCC visibility pop
