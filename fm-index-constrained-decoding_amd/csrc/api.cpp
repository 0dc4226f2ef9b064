// api.cpp -- the extern "C" boundary (include/fmidx.h) over the device index.
//
// Host responsibilities only: argument checking, construction orchestration
// (SA-IS suffix sorting for host-built indexes), persistence, and staging
// of host arguments for the synchronous SWIG-equivalent calls.  Every query
// computes on the GPU through the launchers in query.hip.
#include "fmidx_internal.h"
#include "fileformat.h"
#include "sais.h"
#include "../../include/fmidx.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

namespace fmidx {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

void Index::release() {
  // no kernel on any stream may still read what is freed here (the callers
  // hold the handle's device)
  (void)hipDeviceSynchronize();
  void* ptrs[] = {C, bwt, bwt_view, bm, bm_full, bm_follow, sa, text, ws};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int l = 0; l < kW2MaxLevels; ++l) {
    if (w2_blocks[l]) (void)hipFree(w2_blocks[l]);
    if (w2_sb[l]) (void)hipFree(w2_sb[l]);
    w2_blocks[l] = nullptr;
    w2_sb[l] = nullptr;
  }
  if (w2_Z) (void)hipFree(w2_Z);
  if (E) (void)hipFree(E);
  E = nullptr;
  if (E2) (void)hipFree(E2);
  E2 = nullptr;
  if (cache_bm) (void)hipFree(cache_bm);
  if (cache_tab) (void)hipFree(cache_tab);
  if (trans_tab) (void)hipFree(trans_tab);
  trans_tab = nullptr;
  if (cblock) (void)hipFree(cblock);
  cblock = nullptr;
  trans_entries = trans_dropped = trans_bytes = 0;
  cache_bm = nullptr;
  cache_tab = nullptr;
  cache_nodes = cache_bytes = 0;
  if (D2) (void)hipFree(D2);
  for (void* p : {(void*)mark, (void*)mark_cnt, (void*)sa_samp, (void*)isa_samp})
    if (p) (void)hipFree(p);
  mark = mark_cnt = isa_samp = nullptr;
  sa_samp = nullptr;
  samp_bytes = 0;
  w2_Z = nullptr;
  D2 = nullptr;
  w2_bytes = 0;
  bm_full = nullptr;
  bm_follow = nullptr;
  follow_bytes = 0;
  C = nullptr;
  bwt = nullptr;
  bwt_view = nullptr;
  bm = nullptr;
  sa = nullptr;
  text = nullptr;
  ws = nullptr;
  ws_bytes = 0;
  built = false;
  view = DevView{};
}

}  // namespace fmidx

namespace fmidx {
// process.hip
int launch_processor_step(const DevView& v, const fm_prep_config& cfg, const int64_t* ids, uint64_t B, uint64_t L,
                          uint64_t ld, const int64_t* fdf, uint64_t fdf_len, const float* pow_tab, uint64_t pow_len,
                          const int64_t* prev_ids, uint64_t prev_ld, uint64_t prev_B, const int64_t* prev_state,
                          fm_row_params* rows, uint64_t* mlo, uint64_t* mhi, int64_t* state, uint32_t* status,
                          int64_t* ids_copy, uint64_t copy_ld, bool init_status, hipStream_t s,
                          int32_t* facts = nullptr, uint32_t* rowcase = nullptr);
int launch_prep_finish(const fm_prep_config& cfg, uint64_t B, const int32_t* fsum, const uint32_t* rowcase,
                       const float* pow_tab, uint64_t pow_len, fm_row_params* rows, uint32_t* status, hipStream_t s);
}  // namespace fmidx

using fmidx::set_error;

struct fm_index {
  fmidx::Index idx;
  std::mutex mu;            // serialises host-API staging buffers / workspace
  uint64_t* scratch = nullptr;  // small device scratch for scalar results
  void* stage = nullptr;        // grow-only device staging of the synchronous host-API calls
  void* hstage = nullptr;       // its pinned host mirror (same layout: one copy each way)
  size_t stage_bytes = 0;
  void* dscratch = nullptr;     // device-only scratch of the host API (distinct capacity slots)
  size_t dscratch_bytes = 0;
  // the last use of idx.ws, on whatever stream it ran: every launch that uses
  // the workspace first waits for it (fm_distinct_count_batch runs on the
  // caller's stream, the host API on idx.stream)
  hipEvent_t ws_ev = nullptr;
  bool ws_ev_pending = false;
  // the persistent LF sweep's own workspace (never shared: its tags and counters stay valid
  // between launches), its last use, and the launch epoch (tags of earlier launches never match)
  void* lfp_ws = nullptr;
  size_t lfp_bytes = 0;
  hipEvent_t lfp_ev = nullptr;
  bool lfp_ev_pending = false;
  uint32_t lfp_epoch = 0;
};

namespace {

// Makes the handle's device current for the duration of a call.
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define FM_CHECK_HANDLE(h)                       \
  do {                                           \
    if (!(h)) {                                  \
      set_error("null handle");                  \
      return -1;                                 \
    }                                            \
  } while (0)

#define FM_CHECK_BUILT(h)                        \
  do {                                           \
    FM_CHECK_HANDLE(h);                          \
    if (!(h)->idx.built) {                       \
      set_error("index not initialized");        \
      return -1;                                 \
    }                                            \
  } while (0)

#define FM_GUARD(h)                               \
  DeviceGuard guard_((h)->idx.device);            \
  if (!guard_.ok) {                               \
    set_error("hipSetDevice(%d) failed", (h)->idx.device); \
    return -1;                                    \
  }

// Device staging of the synchronous host-API calls (always under h->mu): one
// grow-only buffer carved into 256-B aligned pieces.  A hipMalloc / hipFree
// pair per call and argument costs tens of us, and hipFree synchronises the
// whole device (other streams' decode steps included).
struct Stage {
  size_t need = 0;
  template <typename T>
  size_t add(size_t count) {
    const size_t off = need;
    need += (std::max<size_t>(count, 1) * sizeof(T) + 255) & ~size_t(255);
    return off;
  }
};

int stage_reserve(fm_index* h, const Stage& st) {
  if (h->stage_bytes >= st.need) return 0;
  // geometric growth: a batch that grows by a few tokens per call (decode) does
  // not reallocate pinned memory (milliseconds per hipHostMalloc) every call
  const size_t bytes = std::max<size_t>({st.need, 2 * h->stage_bytes, (size_t)1 << 20});
  if (h->stage) FM_HIP(hipFree(h->stage));
  if (h->hstage) FM_HIP(hipHostFree(h->hstage));
  h->stage = h->hstage = nullptr;
  h->stage_bytes = 0;
  FM_HIP(hipMalloc(&h->stage, bytes));
  FM_HIP(hipHostMalloc(&h->hstage, bytes, hipHostMallocDefault));
  h->stage_bytes = bytes;
  return 0;
}

template <typename T>
T* stage_at(fm_index* h, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(h->stage) + off);
}

template <typename T>
T* hstage_at(fm_index* h, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(h->hstage) + off);
}

// one copy of the staged span [a, b) each way (pinned: a true async DMA)
int stage_up(fm_index* h, size_t a, size_t b) {
  FM_HIP(hipMemcpyAsync(stage_at<char>(h, a), hstage_at<char>(h, a), b - a, hipMemcpyHostToDevice, h->idx.stream));
  return 0;
}
int stage_down(fm_index* h, size_t a, size_t b) {
  FM_HIP(hipMemcpyAsync(hstage_at<char>(h, a), stage_at<char>(h, a), b - a, hipMemcpyDeviceToHost, h->idx.stream));
  return 0;
}

// Staging / scratch above these sizes is released at the end of the call that
// needed it, so one oversized batch does not pin memory for the handle's life.
constexpr size_t kStageKeep = 64ull << 20;
constexpr size_t kScratchKeep = 256ull << 20;

void stage_trim(fm_index* h) {
  if (h->stage_bytes > kStageKeep) {
    (void)hipFree(h->stage);
    (void)hipHostFree(h->hstage);
    h->stage = h->hstage = nullptr;
    h->stage_bytes = 0;
  }
  if (h->dscratch_bytes > kScratchKeep) {
    (void)hipFree(h->dscratch);
    h->dscratch = nullptr;
    h->dscratch_bytes = 0;
  }
}

int grow_dscratch(fm_index* h, size_t bytes) {
  if (h->dscratch_bytes >= bytes) return 0;
  if (h->dscratch) FM_HIP(hipFree(h->dscratch));
  h->dscratch = nullptr;
  h->dscratch_bytes = 0;
  FM_HIP(hipMalloc(&h->dscratch, bytes));
  h->dscratch_bytes = bytes;
  return 0;
}

// Whether `s` is capturing into a graph.  The handle's workspace is not
// captured: a graph would bake in the pointer of a buffer a later call may
// free and regrow, and the event hand-off between its uses (ws_acquire /
// ws_release) crosses the capture boundary.  (A round-5 run of a workspace
// LF launch inside a captured graph faulted the GPU.)
bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) return false;
  return st != hipStreamCaptureStatusNone;
}

// Workspace of k_distinct (under h->mu): wait for its previous use -- on any
// stream -- before `s` touches it; growing it waits on the host first.
int ws_acquire(fm_index* h, hipStream_t s, size_t bytes) {
  auto& x = h->idx;
  if (!h->ws_ev) FM_HIP(hipEventCreateWithFlags(&h->ws_ev, hipEventDisableTiming));
  if (x.ws_bytes < bytes) {
    if (h->ws_ev_pending) FM_HIP(hipEventSynchronize(h->ws_ev));
    if (x.ws) FM_HIP(hipFree(x.ws));
    x.ws = nullptr;
    x.ws_bytes = 0;
    FM_HIP(hipMalloc(&x.ws, bytes));
    x.ws_bytes = bytes;
  } else if (h->ws_ev_pending) {
    FM_HIP(hipStreamWaitEvent(s, h->ws_ev, 0));
  }
  return 0;
}

// Marks the end of a workspace use enqueued on `s`.
int ws_release(fm_index* h, hipStream_t s) {
  FM_HIP(hipEventRecord(h->ws_ev, s));
  h->ws_ev_pending = true;
  return 0;
}

// Above this many rows the reference's construction entry points
// (initialize / initialize_from_file, fm_index.cpp:33-48) sort on the GPU.
uint64_t gpu_sort_min(const fm_index* h) { return h->idx.opts.gpu_sort_min; }

// Build from a host text T' (+ sentinel already appended): suffix array by
// GPU prefix doubling (n >= the gpu_sort_min option, n < 2^34) or host SA-IS, then
// the device structures; the suffix array is reduced to its samples (locate /
// extract by LF walks) and freed.
int build_from_text(fm_index* h, std::vector<uint32_t>& text) {
  auto& x = h->idx;
  const uint64_t n = text.size();
  x.release();
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&x.bwt), n * 4));
  uint64_t* d_sa = nullptr;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&d_sa), n * 8));
  if (n >= gpu_sort_min(h) && n < (1ull << 34)) {
    uint32_t* d_text = nullptr;
    FM_HIP(hipMalloc(reinterpret_cast<void**>(&d_text), n * 4));
    FM_HIP(hipMemcpyAsync(d_text, text.data(), n * 4, hipMemcpyHostToDevice, x.stream));
    const int rc = fmidx::gpu_suffix_sort(d_text, n, x.bwt, d_sa, x.stream);
    (void)hipStreamSynchronize(x.stream);
    (void)hipFree(d_text);
    if (rc) {
      (void)hipFree(d_sa);
      return -1;
    }
  } else {
    uint32_t maxs = 0;
    for (uint32_t v : text) maxs = std::max(maxs, v);
    std::vector<uint64_t> sa64(n);
    try {
      if (n < (1ull << 31)) {
        std::vector<int32_t> sa;
        fmidx::suffix_array<int32_t>(text.data(), (int64_t)n, maxs + 1, sa);
        for (uint64_t i = 0; i < n; ++i) sa64[i] = (uint64_t)sa[i];
      } else {
        std::vector<int64_t> sa;
        fmidx::suffix_array<int64_t>(text.data(), (int64_t)n, maxs + 1, sa);
        for (uint64_t i = 0; i < n; ++i) sa64[i] = (uint64_t)sa[i];
      }
    } catch (const std::exception& e) {
      (void)hipFree(d_sa);
      set_error("suffix sorting failed: %s", e.what());
      return -1;
    }
    std::vector<uint32_t> bwt(n);
    for (uint64_t i = 0; i < n; ++i) bwt[i] = text[sa64[i] == 0 ? n - 1 : sa64[i] - 1];
    FM_HIP(hipMemcpyAsync(x.bwt, bwt.data(), n * 4, hipMemcpyHostToDevice, x.stream));
    FM_HIP(hipMemcpyAsync(d_sa, sa64.data(), n * 8, hipMemcpyHostToDevice, x.stream));
    FM_HIP(hipStreamSynchronize(x.stream));
  }
  const int rc = fmidx::device_build_samples(&x, d_sa, n, x.stream);
  (void)hipFree(d_sa);
  if (rc) return -1;
  return fmidx::device_build_from_bwt(&x, x.bwt, n, x.stream);
}

int initialize_symbols(fm_index* h, const uint64_t* data, uint64_t n) {
  if (n + 1 > (1ull << 40)) {
    set_error("text too long for the host builder");
    return -1;
  }
  std::vector<uint32_t> text(n + 1);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t v = data[i];
    if (v == 0) {
      set_error("text contains 0 symbol at position %llu (reserved for the sentinel)",
                (unsigned long long)i);
      return -1;
    }
    if (v >= (1ull << fmidx::kMaxLevels)) {
      set_error("symbol %llu at position %llu exceeds 2^%d", (unsigned long long)v,
                (unsigned long long)i, fmidx::kMaxLevels);
      return -1;
    }
    text[i] = (uint32_t)v;
  }
  text[n] = 0;
  return build_from_text(h, text);
}

// Clamped width of a distinct_count query (fm_index.cpp:127-133); 0 = empty.
uint64_t distinct_width(uint64_t lo, uint64_t hi, uint64_t n) {
  if (lo == hi) return 0;
  if (hi > n) hi = n;
  if (lo >= hi) return 0;
  return hi - lo;
}

// Pairs copied back in the call's one device->host copy; a batch with more
// distinct symbols than this takes a second copy for the rest.
constexpr uint64_t kPairsFirstCopy = 1ull << 16;

// Host-staged batched interval_symbols.  Results are compacted on the device
// into a dense CSR (offsets[m + 1] + interleaved (symbol, count) pairs), so
// only the symbols found travel back, not the capacity slots (min(width,
// sigma) per row, ~2 MB for a wide row at a 128k vocabulary).
int host_distinct(fm_index* h, const uint64_t* lows, const uint64_t* highs, uint64_t m,
                  std::vector<uint64_t>& pairs, std::vector<uint64_t>& offsets) {
  auto& x = h->idx;
  std::vector<uint64_t> cap_off(m + 1, 0);
  for (uint64_t i = 0; i < m; ++i)
    cap_off[i + 1] = cap_off[i] + std::min<uint64_t>(distinct_width(lows[i], highs[i], x.n), x.sigma);
  const uint64_t total = cap_off[m];
  const uint64_t first = std::min<uint64_t>(total, kPairsFirstCopy);
  // staged: inputs first, outputs last (one host->device and one device->host copy)
  Stage st;
  const size_t o_lo = st.add<uint64_t>(m), o_hi = st.add<uint64_t>(m), o_cap = st.add<uint64_t>(m + 1),
               o_k = st.add<uint64_t>(m), o_off = st.add<uint64_t>(m + 1), o_pairs = st.add<uint64_t>(2 * first);
  if (stage_reserve(h, st)) return -1;
  // device only: capacity slots (symbols, counts) and the dense pairs
  const uint64_t T = std::max<uint64_t>(total, 1);
  if (grow_dscratch(h, (size_t)T * 32)) return -1;
  uint64_t* d_syms = static_cast<uint64_t*>(h->dscratch);
  uint64_t* d_cnt = d_syms + T;
  uint64_t* d_pairs = d_cnt + T;
  std::memcpy(hstage_at<uint64_t>(h, o_lo), lows, m * 8);
  std::memcpy(hstage_at<uint64_t>(h, o_hi), highs, m * 8);
  std::memcpy(hstage_at<uint64_t>(h, o_cap), cap_off.data(), (m + 1) * 8);
  if (stage_up(h, 0, o_k)) return -1;
  if (ws_acquire(h, x.stream, fmidx::distinct_ws_bytes(total))) return -1;
  if (fmidx::launch_distinct(x.view, stage_at<uint64_t>(h, o_lo), stage_at<uint64_t>(h, o_hi), m,
                             stage_at<uint64_t>(h, o_cap), d_syms, d_cnt, stage_at<uint64_t>(h, o_k), x.ws, total,
                             x.stream))
    return -1;
  if (ws_release(h, x.stream)) return -1;
  if (fmidx::launch_distinct_csr(stage_at<uint64_t>(h, o_k), stage_at<uint64_t>(h, o_cap), d_syms, d_cnt, m,
                                 stage_at<uint64_t>(h, o_off), d_pairs, x.stream))
    return -1;
  if (first)
    FM_HIP(hipMemcpyAsync(stage_at<uint64_t>(h, o_pairs), d_pairs, first * 16, hipMemcpyDeviceToDevice, x.stream));
  if (stage_down(h, o_k, st.need)) return -1;
  FM_HIP(hipStreamSynchronize(x.stream));
  const uint64_t* k = hstage_at<uint64_t>(h, o_k);
  const uint64_t* off = hstage_at<uint64_t>(h, o_off);
  for (uint64_t i = 0; i < m; ++i) {
    if (k[i] == ~0ull) {
      set_error("distinct_count capacity overflow on range %llu", (unsigned long long)i);
      return -1;
    }
  }
  const uint64_t used = off[m];
  offsets.assign(off, off + m + 1);
  pairs.resize(2 * used);
  const uint64_t a = std::min(used, first);
  if (a) std::memcpy(pairs.data(), hstage_at<uint64_t>(h, o_pairs), a * 16);
  if (used > a) {
    FM_HIP(hipMemcpyAsync(pairs.data() + 2 * a, d_pairs + 2 * a, (used - a) * 16, hipMemcpyDeviceToHost, x.stream));
    FM_HIP(hipStreamSynchronize(x.stream));
  }
  return 0;
}

}  // namespace

// Every extern "C" entry catches what the host code may throw (std::bad_alloc
// from a vector sized by a huge request, anything from the standard library)
// and reports it as a status + fm_last_error(): no C++ exception crosses the
// C-ABI into ctypes / cgo / JNI callers.
#define FM_API_BEGIN try {
#define FM_API_CATCH(RET)                          \
  }                                                \
  catch (const std::bad_alloc&) {                  \
    set_error("out of host memory");               \
    RET;                                           \
  }                                                \
  catch (const std::exception& e) {                \
    set_error("C++ exception: %s", e.what());      \
    RET;                                           \
  }                                                \
  catch (...) {                                    \
    set_error("unknown C++ exception");            \
    RET;                                           \
  }
#define FM_API_END FM_API_CATCH(return -1)
#define FM_API_END_VOID FM_API_CATCH(return)

extern "C" {

const char* fm_last_error(void) { return fmidx::g_err.c_str(); }

int fm_device_info(int device, char* buf, size_t cap) {
  FM_API_BEGIN
  hipDeviceProp_t p;
  FM_HIP(hipGetDeviceProperties(&p, device));
  std::snprintf(buf, cap, "%s cu=%d hbm=%zuMB", p.gcnArchName, p.multiProcessorCount,
                (size_t)(p.totalGlobalMem >> 20));
  return 0;
  FM_API_END
}

int fm_create(fm_index** out, int device) {
  FM_API_BEGIN
  if (!out) {
    set_error("null out");
    return -1;
  }
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    set_error("no HIP device available (the FM-index engine has no CPU query path)");
    return -1;
  }
  if (device < 0 || device >= count) {
    set_error("device %d out of range (%d devices)", device, count);
    return -1;
  }
  auto* h = new fm_index();
  h->idx.device = device;
  h->idx.opts = fmidx::build_profile(FM_PROFILE_DEFAULT);
  if (fmidx::apply_build_overrides(h->idx.opts)) {
    delete h;
    return -1;
  }
  DeviceGuard g(device);
  if (!g.ok || hipStreamCreateWithFlags(&h->idx.stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->scratch), 64 * 8) != hipSuccess) {
    set_error("device %d initialisation failed", device);
    delete h;
    return -1;
  }
  *out = h;
  return 0;
  FM_API_END
}

void fm_destroy(fm_index* h) {
  FM_API_BEGIN
  if (!h) return;
  {
    DeviceGuard g(h->idx.device);
    (void)hipDeviceSynchronize();
    h->idx.release();
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->stage) (void)hipFree(h->stage);
    if (h->hstage) (void)hipHostFree(h->hstage);
    if (h->dscratch) (void)hipFree(h->dscratch);
    if (h->ws_ev) (void)hipEventDestroy(h->ws_ev);
    if (h->lfp_ws) (void)hipFree(h->lfp_ws);
    if (h->lfp_ev) (void)hipEventDestroy(h->lfp_ev);
    if (h->idx.stream) (void)hipStreamDestroy(h->idx.stream);
  }
  delete h;
  FM_API_END_VOID
}

int fm_initialize(fm_index* h, const uint64_t* data, uint64_t n) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  if (!data && n) {
    set_error("null data");
    return -1;
  }
  return initialize_symbols(h, data, n);
  FM_API_END
}

int fm_initialize_from_file(fm_index* h, const char* path, int width) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  if (width != 1 && width != 2 && width != 4 && width != 8) {
    set_error("unsupported width %d", width);
    return -1;
  }
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    set_error("cannot open %s", path ? path : "(null)");
    return -1;
  }
  std::vector<unsigned char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const uint64_t n = raw.size() / (uint64_t)width;
  std::vector<uint64_t> data(n);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t v = 0;
    for (int b = width - 1; b >= 0; --b) v = (v << 8) | raw[i * width + b];
    data[i] = v;
  }
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  return initialize_symbols(h, data.data(), n);
  FM_API_END
}

int fm_initialize_from_bwt_device(fm_index* h, const uint32_t* d_bwt, uint64_t n,
                                  const uint64_t* d_sa, const uint32_t* d_text, void* stream) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  auto& x = h->idx;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  FM_HIP(hipStreamSynchronize(s));
  x.release();
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&x.bwt), n * 4));
  FM_HIP(hipMemcpyAsync(x.bwt, d_bwt, n * 4, hipMemcpyDeviceToDevice, x.stream));
  if (d_sa) {
    // locate / extract from SA and ISA samples taken from the caller's SA
    if (fmidx::device_build_samples(&x, d_sa, n, x.stream)) return -1;
  } else if (d_text) {
    // no suffix array: extract_text reads T' directly (locate unavailable)
    FM_HIP(hipMalloc(reinterpret_cast<void**>(&x.text), n * 4));
    FM_HIP(hipMemcpyAsync(x.text, d_text, n * 4, hipMemcpyDeviceToDevice, x.stream));
  }
  FM_HIP(hipStreamSynchronize(x.stream));
  return fmidx::device_build_from_bwt(&x, x.bwt, n, x.stream);
  FM_API_END
}

int fm_initialize_from_text_device(fm_index* h, const uint32_t* d_text, uint64_t n, int keep_sa_text,
                                   void* stream) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  if (!d_text || n == 0) {
    set_error("empty text");
    return -1;
  }
  auto& x = h->idx;
  FM_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  x.release();
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&x.bwt), n * 4));
  uint64_t* d_sa = nullptr;
  if (keep_sa_text) FM_HIP(hipMalloc(reinterpret_cast<void**>(&d_sa), n * 8));
  if (fmidx::gpu_suffix_sort(d_text, n, x.bwt, d_sa, x.stream)) {
    if (d_sa) (void)hipFree(d_sa);
    x.release();
    return -1;
  }
  if (d_sa) {
    const int rc = fmidx::device_build_samples(&x, d_sa, n, x.stream);
    (void)hipFree(d_sa);
    if (rc) return -1;
  }
  return fmidx::device_build_from_bwt(&x, x.bwt, n, x.stream);
  FM_API_END
}

int fm_attach_isa_samples_device(fm_index* h, const uint64_t* d_isa, uint64_t nisa, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  if (!d_isa) {
    set_error("null ISA samples");
    return -1;
  }
  FM_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  return fmidx::device_samples_from_isa(&h->idx, d_isa, nisa, h->idx.stream);
  FM_API_END
}

int fm_suffix_sort_device(const uint32_t* d_text, uint64_t n, uint32_t* d_bwt, uint64_t* d_sa, void* stream) {
  FM_API_BEGIN
  if (!d_text) {
    set_error("null text");
    return -1;
  }
  return fmidx::gpu_suffix_sort(d_text, n, d_bwt, d_sa, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_wt_int_levels_device(const uint32_t* d_bwt, uint64_t n, uint32_t L, uint64_t* d_words, void* stream) {
  FM_API_BEGIN
  if (!d_bwt || !d_words || n == 0) {
    set_error("null or empty input");
    return -1;
  }
  return fmidx::gpu_wt_int_levels(d_bwt, n, L, d_words, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_size(const fm_index* h, uint64_t* out) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  *out = h->idx.n;
  return 0;
  FM_API_END
}

int fm_sigma(const fm_index* h, uint64_t* out) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  *out = h->idx.sigma;
  return 0;
  FM_API_END
}

int fm_backward_search_step(fm_index* h, uint64_t symbol, uint64_t low, uint64_t high,
                            uint64_t out[2]) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  auto& x = h->idx;
  Stage st;
  const size_t o_out = st.add<uint64_t>(2);
  if (stage_reserve(h, st)) return -1;
  if (fmidx::launch_step_raw(x.view, symbol, low, high, stage_at<uint64_t>(h, o_out), x.stream)) return -1;
  if (stage_down(h, o_out, o_out + 16)) return -1;
  FM_HIP(hipStreamSynchronize(x.stream));
  std::memcpy(out, hstage_at<uint64_t>(h, o_out), 16);
  return 0;
  FM_API_END
}

int fm_backward_search_multi(fm_index* h, const uint64_t* query, uint64_t len, uint64_t out[2]) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  auto& x = h->idx;
  Stage st;
  const size_t o_q = st.add<uint64_t>(len);
  const size_t o_out = st.add<uint64_t>(2);
  if (stage_reserve(h, st)) return -1;
  if (len) {
    std::memcpy(hstage_at<uint64_t>(h, o_q), query, len * 8);
    if (stage_up(h, o_q, o_out)) return -1;
  }
  if (fmidx::launch_raw_multi(x.view, stage_at<uint64_t>(h, o_q), len, stage_at<uint64_t>(h, o_out), x.stream))
    return -1;
  if (stage_down(h, o_out, o_out + 16)) return -1;
  FM_HIP(hipStreamSynchronize(x.stream));
  std::memcpy(out, hstage_at<uint64_t>(h, o_out), 16);
  stage_trim(h);
  return 0;
  FM_API_END
}

int fm_distinct_count_multi(fm_index* h, const uint64_t* lows, const uint64_t* highs, uint64_t m,
                            uint64_t* out, uint64_t cap, uint64_t* offsets) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  std::vector<uint64_t> pairs, off;
  const int rc = host_distinct(h, lows, highs, m, pairs, off);
  stage_trim(h);
  if (rc) return -1;
  std::memcpy(offsets, off.data(), (m + 1) * 8);
  if (pairs.size() > cap) {
    set_error("output capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)pairs.size());
    return -2;
  }
  if (!pairs.empty()) std::memcpy(out, pairs.data(), pairs.size() * 8);
  return 0;
  FM_API_END
}

int fm_distinct_count(fm_index* h, uint64_t low, uint64_t high, uint64_t* out, uint64_t cap,
                      uint64_t* k) {
  FM_API_BEGIN
  uint64_t off[2];
  FM_CHECK_BUILT(h);
  // two-call protocol: with too small a buffer report the size and fail
  std::vector<uint64_t> tmp;
  const uint64_t need = 2 * std::min<uint64_t>(distinct_width(low, high, h->idx.n), h->idx.sigma);
  tmp.resize(std::max<uint64_t>(need, 1));
  const int rc = fm_distinct_count_multi(h, &low, &high, 1, tmp.data(), tmp.size(), off);
  if (rc) return rc;
  *k = off[1];
  if (2 * off[1] > cap) {
    set_error("output capacity %llu < %llu", (unsigned long long)cap,
              (unsigned long long)(2 * off[1]));
    return -2;
  }
  std::memcpy(out, tmp.data(), 2 * off[1] * 8);
  return 0;
  FM_API_END
}

int fm_distinct(fm_index* h, uint64_t low, uint64_t high, uint64_t* syms, uint64_t cap, uint64_t* k) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const uint64_t need = 2 * std::min<uint64_t>(distinct_width(low, high, h->idx.n), h->idx.sigma);
  std::vector<uint64_t> tmp(std::max<uint64_t>(need, 1));
  uint64_t kk = 0;
  const int rc = fm_distinct_count(h, low, high, tmp.data(), tmp.size(), &kk);
  if (rc) return rc;
  *k = kk;
  if (kk > cap) {
    set_error("output capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)kk);
    return -2;
  }
  for (uint64_t i = 0; i < kk; ++i) syms[i] = tmp[2 * i];
  return 0;
  FM_API_END
}

int fm_get_range_batch(fm_index* h, const int64_t* tokens, const int64_t* offsets, uint64_t m,
                       int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in,
                       uint64_t* lo_out, uint64_t* hi_out) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  auto& x = h->idx;
  if (m == 0) return 0;
  const uint64_t ntok = (uint64_t)offsets[m];
  const bool starts = lo_in && hi_in;
  // inputs first, outputs last: one host->device and one device->host copy
  Stage st;
  const size_t o_tok = st.add<int64_t>(ntok), o_off = st.add<int64_t>(m + 1), o_li = st.add<uint64_t>(starts ? m : 0),
               o_hi = st.add<uint64_t>(starts ? m : 0), o_lo2 = st.add<uint64_t>(m), o_hi2 = st.add<uint64_t>(m);
  if (stage_reserve(h, st)) return -1;
  if (ntok) std::memcpy(hstage_at<int64_t>(h, o_tok), tokens, ntok * 8);
  std::memcpy(hstage_at<int64_t>(h, o_off), offsets, (m + 1) * 8);
  if (starts) {
    std::memcpy(hstage_at<uint64_t>(h, o_li), lo_in, m * 8);
    std::memcpy(hstage_at<uint64_t>(h, o_hi), hi_in, m * 8);
  }
  if (stage_up(h, 0, o_lo2)) return -1;
  if (fmidx::launch_search(x.view, stage_at<int64_t>(h, o_tok), stage_at<int64_t>(h, o_off), m, shift,
                           starts ? stage_at<uint64_t>(h, o_li) : nullptr, starts ? stage_at<uint64_t>(h, o_hi) : nullptr,
                           stage_at<uint64_t>(h, o_lo2), stage_at<uint64_t>(h, o_hi2), x.stream))
    return -1;
  if (stage_down(h, o_lo2, st.need)) return -1;
  FM_HIP(hipStreamSynchronize(x.stream));
  std::memcpy(lo_out, hstage_at<uint64_t>(h, o_lo2), m * 8);
  std::memcpy(hi_out, hstage_at<uint64_t>(h, o_hi2), m * 8);
  stage_trim(h);
  return 0;
  FM_API_END
}

int fm_locate(fm_index* h, uint64_t row, uint64_t* out) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  auto& x = h->idx;
  if (row >= x.n) {  // fm_index.cpp:170
    *out = ~0ull;
    return 0;
  }
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  if (x.mark) {      // LF walk to the next SA sample (locate.hip)
    Stage st;
    const size_t o_row = st.add<uint64_t>(1), o_out = st.add<uint64_t>(1);
    if (stage_reserve(h, st)) return -1;
    *hstage_at<uint64_t>(h, o_row) = row;
    if (stage_up(h, o_row, o_out)) return -1;
    if (fmidx::launch_locate(x.view, x.samples(), stage_at<uint64_t>(h, o_row), 1, stage_at<uint64_t>(h, o_out),
                             x.stream))
      return -1;
    if (stage_down(h, o_out, o_out + 8)) return -1;
    FM_HIP(hipStreamSynchronize(x.stream));
    *out = *hstage_at<uint64_t>(h, o_out);
    return 0;
  }
  if (!x.sa) {
    set_error("index built without a suffix array: locate unavailable");
    return -1;
  }
  FM_HIP(hipMemcpyAsync(out, x.sa + row, 8, hipMemcpyDeviceToHost, x.stream));
  FM_HIP(hipStreamSynchronize(x.stream));
  return 0;
  FM_API_END
}

int fm_extract_text(fm_index* h, uint64_t begin, uint64_t end, uint64_t* out, uint64_t cap,
                    uint64_t* len) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  auto& x = h->idx;
  *len = 0;
  if (end <= begin) return 0;                // fm_index.cpp:177
  if (end > x.n) end = x.n;                  // :178
  if (end <= begin) {
    // the reference loops (end-begin-1) times in unsigned arithmetic here
    set_error("extract_text: begin %llu >= clamped end %llu (unbounded in the reference)",
              (unsigned long long)begin, (unsigned long long)end);
    return -3;
  }
  if (!x.isa_samp && !x.text) {
    set_error("index built without a suffix array or text: extract_text unavailable");
    return -1;
  }
  const uint64_t L = end - begin;
  *len = L;
  const uint64_t w = std::min(L, cap);
  if (w == 0) return 0;
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  const uint64_t n = x.n;
  if (x.isa_samp) {  // LF walk from isa[end - 1] (locate.hip), out[j] = T'[(end - 2 - j) mod n]
    Stage st;
    const size_t o_b = st.add<uint64_t>(1), o_e = st.add<uint64_t>(1), o_off = st.add<uint64_t>(2),
                 o_out = st.add<uint64_t>(w);
    if (stage_reserve(h, st)) return -1;
    *hstage_at<uint64_t>(h, o_b) = begin;
    *hstage_at<uint64_t>(h, o_e) = end;
    hstage_at<uint64_t>(h, o_off)[0] = 0;
    hstage_at<uint64_t>(h, o_off)[1] = w;
    if (stage_up(h, 0, o_out)) return -1;
    if (fmidx::launch_extract(x.view, x.samples(), stage_at<uint64_t>(h, o_b), stage_at<uint64_t>(h, o_e),
                              stage_at<uint64_t>(h, o_off), 1, stage_at<uint64_t>(h, o_out), x.stream))
      return -1;
    if (stage_down(h, o_out, o_out + w * 8)) return -1;
    FM_HIP(hipStreamSynchronize(x.stream));
    std::memcpy(out, hstage_at<uint64_t>(h, o_out), w * 8);
    stage_trim(h);
    return 0;
  }
  // legacy: read T' (kept when the index was built without a suffix array)
  std::vector<uint32_t> seg;
  uint64_t j = 0;
  uint64_t pos = (end + n - 2) % n;          // position of out[0]
  while (j < w) {
    const uint64_t run = std::min(w - j, pos + 1);  // pos, pos-1, ..., pos-run+1
    seg.resize(run);
    FM_HIP(hipMemcpyAsync(seg.data(), x.text + (pos + 1 - run), run * 4, hipMemcpyDeviceToHost,
                          x.stream));
    FM_HIP(hipStreamSynchronize(x.stream));
    for (uint64_t t = 0; t < run; ++t) out[j + t] = seg[run - 1 - t];
    j += run;
    pos = n - 1;
  }
  return 0;
  FM_API_END
}

// The file layout and its checks: fileformat.h.
static_assert(fmidx::kFileSaRate == fmidx::kSaRate && fmidx::kFileIsaRate == fmidx::kIsaRate &&
                  fmidx::kFileSymBits == fmidx::kMaxSymBits,
              "fileformat.h sampling / symbol constants");

int fm_save(fm_index* h, const char* path) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  auto& x = h->idx;
  const uint64_t n = x.n;
  fmidx::IndexFile f;
  f.n = n;
  f.bwt.resize(n);
  {
    const bool made = !x.bwt && !x.bwt_view;   // materialised for this save only
    const uint32_t* src = nullptr;
    if (fmidx::device_bwt_view(&x, &src)) return -1;
    const hipError_t e = hipMemcpy(f.bwt.data(), src, n * 4, hipMemcpyDeviceToHost);
    if (made) {
      (void)hipFree(x.bwt_view);
      x.bwt_view = nullptr;
    }
    FM_HIP(e);
  }
  if (x.mark) {
    f.mark.resize(fmidx::file_mark_words(n));
    f.samp.resize(fmidx::file_samp_count(n));
    f.isa.resize(fmidx::file_isa_count(n));
    FM_HIP(hipMemcpy(f.mark.data(), x.mark, f.mark.size() * 8, hipMemcpyDeviceToHost));
    FM_HIP(hipMemcpy(f.samp.data(), x.sa_samp, f.samp.size() * 4, hipMemcpyDeviceToHost));
    FM_HIP(hipMemcpy(f.isa.data(), x.isa_samp, f.isa.size() * 8, hipMemcpyDeviceToHost));
  } else if (x.text) {
    f.text.resize(n);
    FM_HIP(hipMemcpy(f.text.data(), x.text, n * 4, hipMemcpyDeviceToHost));
  }
  std::string err;
  if (!fmidx::write_index_file(path, std::move(f), err)) {
    set_error("%s", err.c_str());
    return -1;
  }
  return 0;
  FM_API_END
}

// ---- options (fm_build_options: per handle; fm_tuning: process-wide) ----
}  // extern "C"

namespace {

fmidx::BuildOpts to_internal(const fm_build_options& o) {
  // every field of the profile's, where the caller left the "profile" sentinel (-1 / 0)
  fmidx::BuildOpts x = fmidx::build_profile(o.profile);
  if (o.transitions >= 0) x.transitions = o.transitions;
  if (o.lf_e >= 0) x.lf_e = o.lf_e;
  if (o.lf_e2 >= 0) x.lf_e2 = o.lf_e2;
  if (o.probe_first >= 0) x.probe_first = o.probe_first;
  if (o.keep_bwt >= 0) x.keep_bwt = o.keep_bwt;
  if (o.follow_bitmaps >= 0) x.follow_bitmaps = o.follow_bitmaps;
  if (o.bm_log2 >= 0) x.bm_log2 = o.bm_log2;
  if (o.trans_min > 0) x.trans_min = o.trans_min;
  if (o.cache_min) x.cache_min = o.cache_min;
  if (o.cache_mb) x.cache_mb = o.cache_mb;
  if (o.trans_mb) x.trans_mb = o.trans_mb;
  if (o.gpu_sort_min) x.gpu_sort_min = o.gpu_sort_min;
  return x;
}

void to_public(const fmidx::BuildOpts& x, fm_build_options* o) {
  o->size = sizeof(fm_build_options);
  o->profile = x.profile;
  o->transitions = x.transitions;
  o->lf_e = x.lf_e;
  o->lf_e2 = x.lf_e2;
  o->probe_first = x.probe_first;
  o->keep_bwt = x.keep_bwt;
  o->follow_bitmaps = x.follow_bitmaps;
  o->bm_log2 = x.bm_log2;
  o->trans_min = x.trans_min;
  o->cache_min = x.cache_min;
  o->cache_mb = x.cache_mb;
  o->trans_mb = x.trans_mb;
  o->gpu_sort_min = x.gpu_sort_min;
}

bool valid(const fmidx::BuildOpts& x) {
  auto b = [](int32_t v) { return v == 0 || v == 1; };
  if ((x.profile != FM_PROFILE_DEFAULT && x.profile != FM_PROFILE_COMPACT) || x.transitions < 0 ||
      x.transitions > 2 || !b(x.lf_e) || !b(x.lf_e2) || !b(x.probe_first) || !b(x.keep_bwt) ||
      !b(x.follow_bitmaps) || x.bm_log2 < -1 || x.bm_log2 > 30 || x.cache_min < 2 || x.trans_min < 1) {
    set_error("build options: profile 0/1, transitions 0..2, switches 0/1, bm_log2 -1..30, cache_min >= 2, trans_min >= 1");
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

int fm_build_options_init(fm_build_options* o, int profile) {
  FM_API_BEGIN
  if (!o || (profile != FM_PROFILE_DEFAULT && profile != FM_PROFILE_COMPACT)) {
    set_error("build_options_init: null options or unknown profile %d", profile);
    return -1;
  }
  to_public(fmidx::build_profile(profile), o);
  return 0;
  FM_API_END
}

int fm_set_build_options(fm_index* h, const fm_build_options* o) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  if (!o || o->size != sizeof(fm_build_options)) {
    set_error("set_build_options: null options or size %u != %zu (fm_build_options_init sets it)",
              o ? o->size : 0u, sizeof(fm_build_options));
    return -1;
  }
  fmidx::BuildOpts x = to_internal(*o);
  if (fmidx::apply_build_overrides(x) || !valid(x)) return -1;
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->idx.built) {
    // the options shape the structures a build makes; a built index keeps the ones it was built
    // with, and fm_get_build_options must keep describing them (stats()['follow_bytes'] ...)
    set_error("set_build_options: the index is already built (set them before initialize / load)");
    return -1;
  }
  h->idx.opts = x;
  return 0;
  FM_API_END
}

int fm_get_build_options(const fm_index* h, fm_build_options* o) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  if (!o) {
    set_error("get_build_options: null options");
    return -1;
  }
  to_public(h->idx.opts, o);
  return 0;
  FM_API_END
}

int fm_tuning_init(fm_tuning* t) {
  FM_API_BEGIN
  if (!t) {
    set_error("tuning_init: null tuning");
    return -1;
  }
  const fmidx::Tuning d;
  std::memset(t, 0, sizeof(*t));
  t->size = sizeof(fm_tuning);
  t->lf_group = d.lf_group;
  t->search_group = d.search_group;
  t->dec_threads = d.dec_threads;
  t->mask_slices = d.mask_slices;
  t->lf_group_min = d.lf_group_min;
  t->lf_work = d.lf_work;
  t->lf_gprobe = d.lf_gprobe;
  t->lf_quad = d.lf_quad;
  t->lf_split = d.lf_split;
  t->search_p8 = d.search_p8;
  t->lf_sweep_min = d.lf_sweep_min;
  t->sa_chunk = d.sa_chunk;
  return 0;
  FM_API_END
}

int fm_set_tuning(const fm_tuning* t) {
  FM_API_BEGIN
  if (!t || t->size != sizeof(fm_tuning)) {
    set_error("set_tuning: null tuning or size %u != %zu (fm_tuning_init sets it)", t ? t->size : 0u,
              sizeof(fm_tuning));
    return -1;
  }
  fmidx::Tuning x;
  x.lf_group = t->lf_group;
  x.search_group = t->search_group;
  x.dec_threads = t->dec_threads;
  x.mask_slices = t->mask_slices;
  x.lf_group_min = t->lf_group_min;
  x.lf_work = t->lf_work;
  x.lf_gprobe = t->lf_gprobe;
  x.lf_quad = t->lf_quad;
  x.lf_split = t->lf_split;
  x.search_p8 = t->search_p8;
  x.lf_sweep_min = t->lf_sweep_min;
  x.sa_chunk = t->sa_chunk;
  if (fmidx::set_tuning(x)) return -1;
  fmidx::reload_lf_tuning();
  return 0;
  FM_API_END
}

int fm_get_tuning(fm_tuning* t) {
  FM_API_BEGIN
  if (!t) {
    set_error("get_tuning: null tuning");
    return -1;
  }
  const fmidx::Tuning& x = fmidx::tuning();
  std::memset(t, 0, sizeof(*t));
  t->size = sizeof(fm_tuning);
  t->lf_group = x.lf_group;
  t->search_group = x.search_group;
  t->dec_threads = x.dec_threads;
  t->mask_slices = x.mask_slices;
  t->lf_group_min = x.lf_group_min;
  t->lf_work = x.lf_work;
  t->lf_gprobe = x.lf_gprobe;
  t->lf_quad = x.lf_quad;
  t->lf_split = x.lf_split;
  t->search_p8 = x.search_p8;
  t->lf_sweep_min = x.lf_sweep_min;
  t->sa_chunk = x.sa_chunk;
  return 0;
  FM_API_END
}

int fm_load(fm_index** out, const char* path, int device) { return fm_load_ex(out, path, device, nullptr); }

int fm_load_ex(fm_index** out, const char* path, int device, const fm_build_options* opts) {
  FM_API_BEGIN
  if (!out) {
    set_error("null out");
    return -1;
  }
  *out = nullptr;
  fmidx::IndexFile f;
  std::string err;
  if (!fmidx::read_index_file(path, f, err)) {   // sizes, samples and symbols checked here
    set_error("%s", err.c_str());
    return -1;
  }
  const uint64_t n = f.n;
  fm_index* h = nullptr;
  if (fm_create(&h, device)) return -1;
  if (opts && fm_set_build_options(h, opts)) {
    fm_destroy(h);
    return -1;
  }
  {
    DeviceGuard g(device);
    auto& x = h->idx;
    auto fail = [&]() {
      fm_destroy(h);
      return -1;
    };
    if (hipMalloc(reinterpret_cast<void**>(&x.bwt), n * 4) != hipSuccess) return fail();
    if (hipMemcpy(x.bwt, f.bwt.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return fail();
    if (!f.sa.empty()) {
      uint64_t* d_sa = nullptr;
      if (hipMalloc(reinterpret_cast<void**>(&d_sa), n * 8) != hipSuccess) return fail();
      const bool ok = hipMemcpy(d_sa, f.sa.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess &&
                      fmidx::device_build_samples(&x, d_sa, n, x.stream) == 0;
      (void)hipFree(d_sa);
      if (!ok) return fail();
    } else if (!f.mark.empty()) {
      const uint64_t nwords = f.mark.size(), nsamp = f.samp.size(), nisa = f.isa.size();
      if (hipMalloc(reinterpret_cast<void**>(&x.mark), nwords * 8) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&x.sa_samp), nsamp * 4) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&x.isa_samp), nisa * 8) != hipSuccess)
        return fail();
      if (hipMemcpy(x.mark, f.mark.data(), nwords * 8, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(x.sa_samp, f.samp.data(), nsamp * 4, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(x.isa_samp, f.isa.data(), nisa * 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail();
      if (fmidx::device_finish_samples(&x, n, x.stream)) return fail();
    }
    if (!f.text.empty() && !x.isa_samp) {
      if (hipMalloc(reinterpret_cast<void**>(&x.text), n * 4) != hipSuccess) return fail();
      if (hipMemcpy(x.text, f.text.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return fail();
    }
    if (fmidx::device_build_from_bwt(&x, x.bwt, n, x.stream)) return fail();
  }
  *out = h;
  return 0;
  FM_API_END
}

// ---- batched device entry points ------------------------------------------

int fm_lf_step_batch(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                     const uint64_t* d_lo, const uint64_t* d_hi, uint64_t* d_lo_out,
                     uint64_t* d_hi_out, uint64_t m, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (fmidx::lf_persist(m) && !capturing(s)) {
    std::lock_guard<std::mutex> lk(h->mu);
    const size_t need = fmidx::lf_persist_ws_bytes(m);
    if (!h->lfp_ev) FM_HIP(hipEventCreateWithFlags(&h->lfp_ev, hipEventDisableTiming));
    if (h->lfp_bytes < need) {
      if (h->lfp_ev_pending) FM_HIP(hipEventSynchronize(h->lfp_ev));
      if (h->lfp_ws) FM_HIP(hipFree(h->lfp_ws));
      h->lfp_ws = nullptr;
      h->lfp_bytes = 0;
      FM_HIP(hipMalloc(&h->lfp_ws, need));
      FM_HIP(hipMemsetAsync(h->lfp_ws, 0, need, s));   // counters, error word, tags: zero
      h->lfp_bytes = need;
    } else if (h->lfp_ev_pending) {
      FM_HIP(hipStreamWaitEvent(s, h->lfp_ev, 0));
    }
    if (++h->lfp_epoch == 0) {
      // the epoch wrapped: tags of an old launch could equal a new epoch, and the counter sets
      // alternate by the epoch's parity -- start over from a zeroed workspace at an even epoch
      FM_HIP(hipMemsetAsync(h->lfp_ws, 0, h->lfp_bytes, s));
      h->lfp_epoch = 2;
    }
    const int rc = fmidx::launch_lf_persist(h->idx.view, d_tokens, shift, reset_below, d_lo, d_hi, d_lo_out, d_hi_out,
                                            m, s, h->lfp_ws, h->lfp_bytes, h->lfp_epoch, h->idx.device);
    FM_HIP(hipEventRecord(h->lfp_ev, s));
    h->lfp_ev_pending = true;
    return rc;
  }
  const size_t wsb = fmidx::lf_ws_bytes(m);
  // the worklist variant needs the workspace: under capture the launch takes the workspace-free kernels
  if (!wsb || capturing(s)) return fmidx::launch_lf_step(h->idx.view, d_tokens, shift, reset_below, d_lo, d_hi, d_lo_out, d_hi_out, m, s);
  std::lock_guard<std::mutex> lk(h->mu);     // the workspace and its event are shared (ws_acquire)
  if (ws_acquire(h, s, wsb)) return -1;
  const int rc = fmidx::launch_lf_step(h->idx.view, d_tokens, shift, reset_below, d_lo, d_hi, d_lo_out, d_hi_out, m, s,
                                       h->idx.ws);
  if (ws_release(h, s)) return -1;
  return rc;
  FM_API_END
}

int fm_backward_search_batch(fm_index* h, const int64_t* d_tokens, const int64_t* d_offsets,
                             uint64_t m, int64_t shift, const uint64_t* d_lo_in,
                             const uint64_t* d_hi_in, uint64_t* d_lo_out, uint64_t* d_hi_out,
                             void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_search(h->idx.view, d_tokens, d_offsets, m, shift, d_lo_in, d_hi_in,
                              d_lo_out, d_hi_out, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_allowed_mask_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m,
                          uint8_t* d_mask, uint64_t ld, uint64_t vocab, int64_t shift, int packed,
                          void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_mask(h->idx.view, d_lo, d_hi, m, d_mask, ld, vocab, shift, packed,
                            reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_decode_step_batch(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                         const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out,
                         uint64_t* d_hi_out, uint64_t m, uint8_t* d_mask, uint64_t ld,
                         uint64_t vocab, int packed, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_decode(h->idx.view, d_tokens, shift, reset_below, d_lo_in, d_hi_in, d_lo_out,
                              d_hi_out, m, d_mask, ld, vocab, packed, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_decode_step_payload(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                           const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out, uint64_t* d_hi_out,
                           uint64_t m, uint32_t* d_payload, uint64_t cap_words, uint64_t vocab,
                           uint32_t* d_payload_alt, const uint32_t* d_step, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_decode_payload(h->idx.view, d_tokens, shift, reset_below, d_lo_in, d_hi_in, d_lo_out, d_hi_out,
                                      m, d_payload, cap_words, vocab, d_payload_alt, d_step,
                                      reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_decode_step_payload_signal(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                                  const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out,
                                  uint64_t* d_hi_out, uint64_t m, uint32_t* d_payload, uint64_t cap_words,
                                  uint64_t vocab, uint32_t* d_payload_alt, uint32_t* d_step,
                                  const uint64_t* d_flag_ptrs, uint64_t world, uint32_t* d_done, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  if (!d_step || !d_done || !d_payload_alt) {
    set_error("decode_step_payload_signal: the step counter, the done counter and both payload buffers");
    return -1;
  }
  return fmidx::launch_decode_payload(h->idx.view, d_tokens, shift, reset_below, d_lo_in, d_hi_in, d_lo_out, d_hi_out,
                                      m, d_payload, cap_words, vocab, d_payload_alt, d_step,
                                      reinterpret_cast<hipStream_t>(stream), d_flag_ptrs, world, d_done);
  FM_API_END
}

int fm_distinct_count_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m,
                            const uint64_t* d_cap_off, uint64_t total_cap, uint64_t* d_syms,
                            uint64_t* d_counts, uint64_t* d_k, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (capturing(s)) {
    set_error("fm_distinct_count_batch: not capturable (it uses the handle's workspace); launch it eagerly");
    return -1;
  }
  if (ws_acquire(h, s, fmidx::distinct_ws_bytes(total_cap))) return -1;
  if (fmidx::launch_distinct(h->idx.view, d_lo, d_hi, m, d_cap_off, d_syms, d_counts, d_k, h->idx.ws, total_cap, s))
    return -1;
  return ws_release(h, s);
  FM_API_END
}

int fm_apply_boosts(int dtype, const void* d_scores, void* d_out, uint64_t B, uint64_t V,
                    uint64_t ld_scores, uint64_t ld_out, const uint32_t* d_bits, uint64_t ld_bits,
                    const uint32_t* d_unigram_bits, const fm_row_params* d_rows, int64_t eos,
                    void* stream) {
  FM_API_BEGIN
  static_assert(sizeof(fm_row_params) == 32, "fm_row_params layout");
  return fmidx::launch_epilogue(dtype, d_scores, d_out, B, V, ld_scores, ld_out, d_bits, ld_bits,
                                d_unigram_bits, d_rows, eos, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_locate_batch(fm_index* h, const uint64_t* d_rows, uint64_t m, uint64_t* d_out, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_locate(h->idx.view, h->idx.samples(), d_rows, m, d_out, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_extract_batch(fm_index* h, const uint64_t* d_begin, const uint64_t* d_end, const uint64_t* d_off, uint64_t m,
                     uint64_t* d_out, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_extract(h->idx.view, h->idx.samples(), d_begin, d_end, d_off, m, d_out,
                               reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_stats_mem(const fm_index* h, uint64_t* e_bytes, uint64_t* sample_bytes, uint64_t* total_bytes) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const auto& x = h->idx;
  const uint64_t e = (x.E ? x.n * 8 : 0) + (x.E2 ? x.n * 4 : 0);
  const uint64_t K = (1ull << x.L) + 1;
  if (e_bytes) *e_bytes = e;
  if (sample_bytes) *sample_bytes = x.samp_bytes;
  if (total_bytes)
    // (cache_bytes already holds the transition table: build_transitions adds it there)
    *total_bytes = (x.bwt ? x.n * 4 : 0) + x.bm_bytes + x.follow_bytes +
                   (x.bm_full ? (uint64_t)x.view.bm_words * 4 : 0) + x.w2_bytes + e + x.cache_bytes + x.samp_bytes +
                   (x.sa ? x.n * 8 : 0) + (x.text ? x.n * 4 : 0) + 2 * K * 8;
  return 0;
  FM_API_END
}

int fm_stats(const fm_index* h, uint64_t* levels, uint64_t* wm_bytes, uint64_t* bwt_bytes,
             uint64_t* bitmap_bytes, uint64_t* bitmap_block) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const auto& x = h->idx;
  if (levels) *levels = x.view.NL2;   // the one wavelet matrix: the 2-level one
  if (wm_bytes) *wm_bytes = x.w2_bytes;
  if (bwt_bytes) *bwt_bytes = x.bwt ? x.n * 4 : 0;
  if (bitmap_bytes) *bitmap_bytes = x.bm_bytes + x.follow_bytes + (x.bm_full ? (uint64_t)x.view.bm_words * 4 : 0);
  if (bitmap_block) *bitmap_block = x.view.bm_levels ? (1ull << x.view.bm_log2) : 0;
  return 0;
  FM_API_END
}

int fm_stats_ex(const fm_index* h, uint64_t* w2_levels, uint64_t* w2_bytes, uint64_t* cache_nodes,
                uint64_t* cache_bytes, uint64_t* cache_min) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const auto& x = h->idx;
  if (w2_levels) *w2_levels = x.view.NL2;
  if (w2_bytes) *w2_bytes = x.w2_bytes;
  if (cache_nodes) *cache_nodes = x.cache_nodes;
  if (cache_bytes) *cache_bytes = x.cache_bytes;
  if (cache_min) *cache_min = x.view.cache_mask ? x.view.cache_min : 0;
  return 0;
  FM_API_END
}

int fm_stats_trans(const fm_index* h, uint64_t* entries, uint64_t* dropped, uint64_t* bytes) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const auto& x = h->idx;
  if (entries) *entries = x.trans_entries;
  if (dropped) *dropped = x.trans_dropped;
  if (bytes) *bytes = x.trans_bytes;
  return 0;
  FM_API_END
}

int fm_stats_trans_complete(const fm_index* h, uint32_t* complete) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  if (complete) *complete = (h->idx.view.probe_first & fmidx::kProbeComplete) ? 1u : 0u;
  return 0;
  FM_API_END
}

int fm_cache_lookup_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m, uint8_t* d_out,
                          void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_cache_probe(h->idx.view, d_lo, d_hi, m, d_out, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_processor_step(fm_index* h, const fm_prep_config* cfg, const int64_t* d_ids, uint64_t B, uint64_t L,
                      uint64_t ld_ids, const int64_t* d_fdf, uint64_t fdf_len, const float* d_pow, uint64_t pow_len,
                      const int64_t* d_prev_ids, uint64_t prev_ld, uint64_t prev_B, const int64_t* d_prev_state,
                      fm_row_params* d_rows, uint64_t* d_mask_lo, uint64_t* d_mask_hi, int64_t* d_state,
                      uint32_t* d_status, void* stream) {
  FM_API_BEGIN
  static_assert(sizeof(fm_prep_config) == 192, "fm_prep_config layout");
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  if (!cfg) {
    set_error("null config");
    return -1;
  }
  return fmidx::launch_processor_step(h->idx.view, *cfg, d_ids, B, L, ld_ids, d_fdf, fdf_len, d_pow, pow_len,
                                      d_prev_ids, prev_ld, prev_B, d_prev_state, d_rows, d_mask_lo, d_mask_hi,
                                      d_state, d_status, nullptr, 0, true, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_processor_call(fm_index* h, const fm_prep_config* cfg, const fm_processor_args* a, void* stream) {
  FM_API_BEGIN
  static_assert(sizeof(fm_processor_args) == 248, "fm_processor_args layout");
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  if (!cfg || !a) {
    set_error("null config or arguments");
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 1. row bookkeeping + pattern ranges
  if (fmidx::launch_processor_step(h->idx.view, *cfg, a->ids, a->B, a->L, a->ld, a->fdf, a->fdf_len, a->pow_tab,
                                   a->pow_len, a->prev_ids, a->prev_ld, a->prev_B, a->prev_state, a->rows, a->mask_lo,
                                   a->mask_hi, a->state, a->status, a->ids_copy, a->copy_ld,
                                   a->status_host || a->status_event, s))
    return -1;
  // the status right behind the bookkeeping: the host waits on status_event (not on the whole
  // call) to learn whether the device path holds, while the mask and the epilogue run
  if (a->status_host) FM_HIP(hipMemcpyAsync(a->status_host, a->status, 16, hipMemcpyDeviceToHost, s));
  if (a->status_event) FM_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(a->status_event), s));
  // 2. the allowed bits of the rows that need them (empty ranges give zero rows)
  if (a->B && fmidx::launch_mask(h->idx.view, a->mask_lo, a->mask_hi, a->B, reinterpret_cast<uint8_t*>(a->bits),
                                 a->bits_ld * 4, a->V, cfg->shift, 1, s))
    return -1;
  // 3. scores + mask
  if (a->B && fmidx::launch_epilogue(a->dtype, a->scores, a->out, a->B, a->V, a->ld_scores, a->ld_out, a->bits,
                                     a->bits_ld, a->unigram_bits, a->rows, a->eos, s))
    return -1;
  return 0;
  FM_API_END
}

int fm_processor_shard_prep(fm_index* h, const fm_prep_config* cfg, const fm_processor_args* a, int32_t* d_facts,
                            uint32_t* d_rowcase, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  if (!cfg || !a || !d_facts || !d_rowcase) {
    set_error("null config, arguments, facts or rowcase");
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 1. row bookkeeping + this shard's ranges and facts
  if (fmidx::launch_processor_step(h->idx.view, *cfg, a->ids, a->B, a->L, a->ld, a->fdf, a->fdf_len, a->pow_tab,
                                   a->pow_len, a->prev_ids, a->prev_ld, a->prev_B, a->prev_state, a->rows, a->mask_lo,
                                   a->mask_hi, a->state, a->status, a->ids_copy, a->copy_ld, true, s, d_facts,
                                   d_rowcase))
    return -1;
  // 2. this shard's allowed bits of every searched row (to be ORed over the shards)
  if (a->B && fmidx::launch_mask(h->idx.view, a->mask_lo, a->mask_hi, a->B, reinterpret_cast<uint8_t*>(a->bits),
                                 a->bits_ld * 4, a->V, cfg->shift, 1, s))
    return -1;
  return 0;
  FM_API_END
}

int fm_processor_shard_finish(const fm_prep_config* cfg, const fm_processor_args* a, const int32_t* d_facts_sum,
                              const uint32_t* d_rowcase, const uint32_t* d_bits, uint64_t bits_ld, void* stream) {
  FM_API_BEGIN
  if (!cfg || !a) {
    set_error("null config or arguments");
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (fmidx::launch_prep_finish(*cfg, a->B, d_facts_sum, d_rowcase, a->pow_tab, a->pow_len, a->rows, a->status, s))
    return -1;
  if (a->status_host) FM_HIP(hipMemcpyAsync(a->status_host, a->status, 16, hipMemcpyDeviceToHost, s));
  if (a->status_event) FM_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(a->status_event), s));
  if (a->B && fmidx::launch_epilogue(a->dtype, a->scores, a->out, a->B, a->V, a->ld_scores, a->ld_out, d_bits,
                                     bits_ld, a->unigram_bits, a->rows, a->eos, s))
    return -1;
  return 0;
  FM_API_END
}

int fm_or_bits(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t words_per_row,
               uint64_t vocab, void* d_out, uint64_t ld_out, int unpack, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_or_bits(d_parts, nparts, part_stride, B, words_per_row, vocab, d_out, ld_out, unpack,
                               reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_payload_capacity(uint64_t B, uint64_t vocab, uint64_t* words) {
  FM_API_BEGIN
  if (!words) {
    set_error("null out");
    return -1;
  }
  *words = fmidx::shard_payload_capacity(B, vocab);
  return 0;
  FM_API_END
}

int fm_shard_pack(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t B, const uint32_t* d_bits,
                  uint64_t ldw, uint64_t vocab, uint32_t* d_payload, uint64_t cap_words, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_shard_pack(h->idx.view, d_lo, d_hi, B, d_bits, ldw, vocab, nullptr, d_payload, cap_words,
                                  reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_pack_facts(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t B, const uint32_t* d_bits,
                        uint64_t ldw, uint64_t vocab, const int32_t* d_facts, uint32_t* d_payload, uint64_t cap_words,
                        void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  return fmidx::launch_shard_pack(h->idx.view, d_lo, d_hi, B, d_bits, ldw, vocab, d_facts, d_payload, cap_words,
                                  reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_or_rows(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t vocab,
                     int64_t shift, void* d_out, uint64_t ld_out, int unpack, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_shard_or_rows(d_parts, nparts, part_stride, B, vocab, shift, d_out, ld_out, unpack, nullptr,
                                     reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_or_rows_facts(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t vocab,
                           int64_t shift, void* d_out, uint64_t ld_out, int unpack, int32_t* d_facts_out,
                           void* stream) {
  FM_API_BEGIN
  return fmidx::launch_shard_or_rows(d_parts, nparts, part_stride, B, vocab, shift, d_out, ld_out, unpack, d_facts_out,
                                     reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_or_rows_peers(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                           uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_shard_or_rows_peers(d_part_ptrs, nparts, cap_words, B, vocab, shift, d_out, ld_out, unpack,
                                           nullptr, nullptr, 0, nullptr, nullptr, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_or_rows_peers_wait(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                                uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack,
                                const uint32_t* d_flags, const uint32_t* d_step, uint32_t spins, uint32_t* err,
                                void* stream) {
  FM_API_BEGIN
  if (!d_flags) {
    set_error("shard_or_rows_peers_wait: null flags");
    return -1;
  }
  return fmidx::launch_shard_or_rows_peers(d_part_ptrs, nparts, cap_words, B, vocab, shift, d_out, ld_out, unpack,
                                           d_flags, d_step, spins, err, nullptr, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_shard_or_rows_peers_facts(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                                 uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack,
                                 const uint32_t* d_flags, const uint32_t* d_step, uint32_t spins, uint32_t* err,
                                 int32_t* d_facts_out, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_shard_or_rows_peers(d_part_ptrs, nparts, cap_words, B, vocab, shift, d_out, ld_out, unpack,
                                           d_flags, d_step, spins, err, d_facts_out,
                                           reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

static_assert(sizeof(fm_peer_step) == 168 && offsetof(fm_peer_step, reset_below) == 160,
              "fm_peer_step: fmidx/sharding.py's FmPeerStep mirrors this layout");
int fm_peer_flags_step(fm_index* h, const fm_peer_step* p, const int64_t* d_tokens, int sync, void* stream) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  if (!p || !p->d_step || !p->d_done || !p->d_payload_alt || !p->d_flags || !p->d_part_ptrs) {
    set_error("peer_flags_step: the step counter, the done counter, both payload buffers, the flags and the parts");
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (fmidx::launch_decode_payload(h->idx.view, d_tokens, p->shift, p->reset_below, p->d_lo, p->d_hi, p->d_lo, p->d_hi,
                                   p->m, p->d_payload, p->cap_words, p->vocab, p->d_payload_alt, p->d_step, s,
                                   p->d_flag_ptrs, p->world, p->d_done))
    return -1;
  if (fmidx::launch_shard_or_rows_peers(p->d_part_ptrs, p->nparts, p->cap_words, p->m, p->vocab, p->shift, p->d_out,
                                        p->ld_out, p->unpack, p->d_flags, p->d_step, p->spins, p->err, nullptr, s))
    return -1;
  if (!sync || capturing(s)) return 0;
  FM_HIP(hipStreamSynchronize(s));
  return (p->err && *reinterpret_cast<volatile uint32_t*>(p->err)) ? 1 : 0;
  FM_API_END
}

int fm_lf_persist_status(fm_index* h, uint32_t* err) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  *err = 0;
  if (!h->lfp_ws) return 0;
  if (h->lfp_ev_pending) FM_HIP(hipEventSynchronize(h->lfp_ev));
  FM_HIP(hipMemcpy(err, static_cast<char*>(h->lfp_ws) + fmidx::lf_persist_err_offset(), 4, hipMemcpyDeviceToHost));
  return 0;
  FM_API_END
}

int fm_peer_signal(const uint64_t* d_flag_ptrs, uint64_t world, uint32_t* d_step, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_peer_signal(d_flag_ptrs, world, d_step, reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_host_mapped_alloc(uint64_t bytes, void** out) {
  FM_API_BEGIN
  if (!out || !bytes) {
    set_error("host_mapped_alloc: null output or zero bytes");
    return -1;
  }
  *out = nullptr;
  // coherent (fine-grained) mapped host memory: a kernel's system-scope store lands in host
  // memory, where the host reads it without a copy or a synchronisation
  FM_HIP(hipHostMalloc(out, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(*out, 0, bytes);
  return 0;
  FM_API_END
}

int fm_host_mapped_free(void* p) {
  FM_API_BEGIN
  if (p) FM_HIP(hipHostFree(p));
  return 0;
  FM_API_END
}

int fm_ipc_handle(const void* d_ptr, uint8_t* handle, uint64_t* offset) {
  FM_API_BEGIN
  if (!d_ptr || !handle || !offset) {
    set_error("ipc_handle: null argument");
    return -1;
  }
  // the handle names the whole allocation (torch's caching allocator hands out pieces of
  // larger blocks): the peer adds the offset to the base it maps
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  FM_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(d_ptr)));
  hipIpcMemHandle_t hd;
  FM_HIP(hipIpcGetMemHandle(&hd, base));
  static_assert(sizeof(hd) == FM_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");
  std::memcpy(handle, &hd, sizeof(hd));
  *offset = (uint64_t)(static_cast<const char*>(d_ptr) - static_cast<const char*>(base));
  return 0;
  FM_API_END
}

int fm_ipc_open(const uint8_t* handle, void** d_base) {
  FM_API_BEGIN
  if (!handle || !d_base) {
    set_error("ipc_open: null argument");
    return -1;
  }
  hipIpcMemHandle_t hd;
  std::memcpy(&hd, handle, sizeof(hd));
  *d_base = nullptr;
  FM_HIP(hipIpcOpenMemHandle(d_base, hd, hipIpcMemLazyEnablePeerAccess));
  return 0;
  FM_API_END
}

int fm_ipc_close(void* d_base) {
  FM_API_BEGIN
  if (!d_base) return 0;
  FM_HIP(hipIpcCloseMemHandle(d_base));
  return 0;
  FM_API_END
}

int fm_probe_gather(const void* d_buf, uint64_t bytes, int chase, uint64_t loads, uint32_t threads,
                    uint64_t* d_sink, void* stream) {
  FM_API_BEGIN
  return fmidx::launch_probe_gather(d_buf, bytes, chase, loads, threads, d_sink,
                                    reinterpret_cast<hipStream_t>(stream));
  FM_API_END
}

int fm_device_bwt(const fm_index* h, const uint32_t** out) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  // the kept BWT, or a copy materialised from E (held by the handle; not a query structure)
  auto* hm = const_cast<fm_index*>(h);
  std::lock_guard<std::mutex> lk(hm->mu);
  return fmidx::device_bwt_view(&hm->idx, out);
  FM_API_END
}

int fm_release_bwt_view(fm_index* h) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  FM_GUARD(h);
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->idx.bwt_view) {
    // the caller's pointers into it are dead from here: synchronise the device first, so no
    // stream-ordered reader of it is still in flight
    FM_HIP(hipDeviceSynchronize());
    FM_HIP(hipFree(h->idx.bwt_view));
    h->idx.bwt_view = nullptr;
  }
  return 0;
  FM_API_END
}

int fm_stats_views(const fm_index* h, uint64_t* bwt_view_bytes) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  if (bwt_view_bytes) *bwt_view_bytes = h->idx.bwt_view ? h->idx.n * 4 : 0;
  return 0;
  FM_API_END
}

int fm_device_struct(const fm_index* h, int which, const void** out, uint64_t* bytes) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  const auto& x = h->idx;
  const void* p = nullptr;
  uint64_t b = 0;
  switch (which) {
    case 0: p = x.bwt; b = x.bwt ? x.n * 4 : 0; break;   // null once freed (E holds the symbols)
    case 1: p = x.E; b = x.E ? x.n * 8 : 0; break;
    case 2: p = x.trans_tab; b = x.trans_bytes; break;
    case 3: p = x.cache_bm; b = x.cache_bm ? x.cache_nodes * (uint64_t)x.view.bm_words * 4 : 0; break;
    case 4: p = x.w2_blocks[0]; b = x.w2_blocks[0] ? x.view.w2[0].blk_bytes * ((x.n + fmidx::kW2Blk - 1) / fmidx::kW2Blk) : 0; break;
    default: fmidx::set_error("fm_device_struct: unknown structure %d", which); return -1;
  }
  *out = p;
  *bytes = p ? b : 0;
  return 0;
  FM_API_END
}

#ifdef FMIDX_STAMPS
// Diagnostic build only (not part of include/fmidx.h): per-workgroup phase
// stamps of the decode kernel go to d_buf (16 uint64 per workgroup: 8 stamps + the row served), or off.
int fm_debug_set_stamps(fm_index* h, uint64_t* d_buf) {
  FM_API_BEGIN
  FM_CHECK_BUILT(h);
  h->idx.view.stamps = d_buf;
  return 0;
  FM_API_END
}
#endif

int fm_reload_tuning(void) {
  FM_API_BEGIN
  // the library defaults with the FMIDX_TUNING overrides on top
  if (fmidx::set_tuning(fmidx::Tuning{})) return -1;
  fmidx::reload_lf_tuning();
  return 0;
  FM_API_END
}

int fm_synchronize(fm_index* h) {
  FM_API_BEGIN
  FM_CHECK_HANDLE(h);
  FM_GUARD(h);
  FM_HIP(hipDeviceSynchronize());
  return 0;
  FM_API_END
}

}  // extern "C"
