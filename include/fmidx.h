/*
 * fmidx.h -- C-ABI of the MI355X-native FM-index engine (libfmidx.so).
 *
 * This is the drop-in boundary that replaces the SWIG module
 * ``cpp_modules.fm_index`` (reference: cpp_modules_linux/fm_index.{hpp,cpp,i}).
 * Every SWIG method of class ``FMIndex`` has an ``fm_*`` equivalent on an
 * opaque handle; in addition the batched hot-path entry points take DEVICE
 * pointers and a ``hipStream_t`` (passed as ``void*``) so a logits processor
 * can build a (rows x vocab) allowed-token mask with no host round trip.
 *
 * Conventions
 *  - Every function returns an int status: 0 = ok, < 0 = error; the message
 *    of the last error on the calling thread is in fm_last_error().
 *  - Symbols are the reference's ``char_type`` (unsigned long, fm_index.hpp:22):
 *    token id + SHIFT (index.py:16); the batched entry points instead take
 *    int64 token ids plus a ``shift`` so they can read ``input_ids`` directly.
 *  - Ranges are half-open [low, high) unless a comment says "inclusive"
 *    (fm_index.cpp:67 takes an inclusive high, and returns a half-open one).
 *  - Host-pointer functions are synchronous.  Device-pointer functions are
 *    stream-ordered on ``stream`` (NULL = the legacy default stream) and never
 *    allocate or synchronise, so they can be captured into a hipGraph, except
 *    where noted (workspace growth on first use).
 *  - There is no CPU query path: every query executes on the GPU that holds
 *    the index.  Construction (suffix sorting) runs on the host or, for the
 *    device-build entry points, on the GPU.
 */
#ifndef FMIDX_H_
#define FMIDX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fm_index fm_index;

/* ---- lifecycle / errors ------------------------------------------------ */

/* Last error message of the calling thread ("" if none). */
const char* fm_last_error(void);

/* Library / device info: writes a short string (arch, CU count). */
int fm_device_info(int device, char* buf, size_t cap);

/* FMIndex::FMIndex()  -- fm_index.cpp:27-29.  Binds the handle to ``device``. */
int fm_create(fm_index** out, int device);

/* FMIndex::~FMIndex() -- fm_index.cpp:31 (frees host and device memory). */
void fm_destroy(fm_index* h);

/* ---- options ----------------------------------------------------------- */

/* Which acceleration structures an index is built with (no reference
 * counterpart: sdsl's csa_wt_int<> has one layout, fm_index.hpp:36).  Set on
 * a handle before any fm_initialize* (or give it to fm_load_ex); the values
 * in force are fm_get_build_options'.  fm_build_options_init fills a profile:
 *   FM_PROFILE_DEFAULT -- every structure (89.1 GiB at n = 4.5e9, V = 128256;
 *     13.8 us per cold B = 256 decode step);
 *   FM_PROFILE_COMPACT -- transitions to cached children only, no E array,
 *     the transition probe issued with the descent (54.3 GiB there, +24 % cold).
 * Then change fields as needed.  An int field of -1 or a size field of 0 means
 * "the profile's value".  The environment variable FMIDX_BUILD_OPTIONS
 * ("key=value,...", keys = the field names) overrides the fields at
 * fm_create / fm_set_build_options time (measurement runs).
 * fm_set_build_options returns -1 once the handle's index is built (a built
 * index keeps, and fm_get_build_options reports, the options it was built with). */
#define FM_PROFILE_DEFAULT 0
#define FM_PROFILE_COMPACT 1
typedef struct fm_build_options {
  uint32_t size;            /* sizeof(fm_build_options) (set by fm_build_options_init) */
  int32_t profile;          /* FM_PROFILE_* */
  int32_t transitions;      /* transition table: 0 none, 1 cached children only, 2 every child of a cached range */
  int32_t lf_e;             /* 1: the E array (LF(i) | BWT[i]: one scan for the LF step of a narrow range) */
  int32_t lf_e2;            /* 1: BWT[LF(i)] beside E (measured neutral: 0) */
  int32_t probe_first;      /* 1: a cached range's LF step waits for its transition probe before any rank load */
  int32_t keep_bwt;         /* 1: keep the plain BWT although E holds its symbols */
  int32_t follow_bitmaps;   /* 1: a bitmap per symbol of its C-block (0: the range cache holds the wide ones) */
  int32_t bm_log2;          /* aligned bitmap block, log2 rows; -1: by n (16 from 2^31 rows, 14 from 2^26, 12 below) */
  int32_t trans_min;        /* transitions = 2: only the children of >= trans_min occurrences (1); <= 0: the profile's */
  uint64_t cache_min;       /* range-bitmap cache: every SA range of >= cache_min rows reachable from the root (4096) */
  uint64_t cache_mb;        /* its budget, MiB (48 GiB) */
  uint64_t trans_mb;        /* the transition table's budget, MiB (72 GiB; past it: cached children only) */
  uint64_t gpu_sort_min;    /* fm_initialize / fm_initialize_from_file sort on the GPU from this many rows (2^20) */
} fm_build_options;
int fm_build_options_init(fm_build_options* o, int profile);
int fm_set_build_options(fm_index* h, const fm_build_options* o);
int fm_get_build_options(const fm_index* h, fm_build_options* o);

/* Launch tuning of the query kernels, process-wide (the measured defaults of
 * DESIGN.md §4 from fm_tuning_init).  fm_set_tuning while no launch is being
 * issued; FMIDX_TUNING ("key=value,...") overrides it for measurement runs,
 * and fm_reload_tuning restores the defaults with those overrides. */
typedef struct fm_tuning {
  uint32_t size;            /* sizeof(fm_tuning) (set by fm_tuning_init) */
  uint32_t lf_group;        /* lanes per row of LF launches above lf_group_min rows: 1, 2, 4, 8, 16; 64 never groups (2) */
  uint32_t search_group;    /* the same for get_range launches (1) */
  uint32_t dec_threads;     /* decode workgroup size 256 / 512 / 1024; 0 = by batch (1024 up to 256 rows, 256 beyond) */
  uint32_t mask_slices;     /* vocabulary slices per decode row; 0 = by the resident-wave budget */
  uint32_t reserved;
  uint64_t lf_group_min;    /* grouped LF / get_range kernels above this many rows (8192) */
  int32_t lf_work;          /* -1: the in-wave sweep from lf_sweep_min rows, else the grouped kernel; 0 grouped only;
                               4: the persistent sweep from lf_sweep_min rows (heads, then a shared tail-queue drain);
                               1 sweep + worklist tail (not inside a captured graph: the grouped kernel
                               there); 2 in-wave sweep whenever grouped */
  int32_t lf_gprobe;        /* groups of >= 4 lanes probe the transition table themselves (1) */
  int32_t lf_quad;          /* two-lane LF launches settle wide rows four at a time first (1) */
  int32_t lf_split;         /* two-pass LF launch, cheap rows then wide rows (0: measured slower) */
  int32_t search_p8;        /* get_range probes cached wide rows eight per round trip (1) */
  int32_t reserved2;
  uint64_t lf_sweep_min;    /* see lf_work (2^18) */
  uint64_t sa_chunk;        /* suffix sorter: rows per sort chunk (2^29) */
} fm_tuning;
int fm_tuning_init(fm_tuning* t);
int fm_set_tuning(const fm_tuning* t);
int fm_get_tuning(fm_tuning* t);

/* ---- construction ------------------------------------------------------ */

/* FMIndex::initialize(const vector<char_type>&) -- fm_index.cpp:33-41.
 * ``data`` is T' (already reversed / shifted by index.py:47-53) WITHOUT the
 * sentinel; a 0 symbol is an error (sdsl construct rejects it).  Builds the
 * suffix array on the host (SA-IS), then the BWT, wavelet matrix, C table,
 * range bitmaps and SA/text arrays on the device. */
int fm_initialize(fm_index* h, const uint64_t* data, uint64_t n);

/* FMIndex::initialize_from_file(string, int width) -- fm_index.cpp:43-48:
 * ``width``-byte little-endian unsigned integers (index.py:63 writes '<l'). */
int fm_initialize_from_file(fm_index* h, const char* path, int width);

/* Device build from a finished BWT already resident in HBM (no host copy):
 * ``d_bwt`` holds n uint32 symbols with exactly one 0 (the sentinel row).
 * Optional ``d_sa`` (n uint64, may be NULL) enables fm_locate and
 * ``d_text`` (n uint32 = T' with sentinel, may be NULL) enables extract.
 * The buffers are copied; the caller keeps ownership. */
int fm_initialize_from_bwt_device(fm_index* h, const uint32_t* d_bwt, uint64_t n,
                                  const uint64_t* d_sa, const uint32_t* d_text,
                                  void* stream);

/* Index construction on the GPU from a device-resident T' (replaces sdsl
 * construct_im / construct, fm_index.cpp:33-48, whose divsufsort runs on the
 * host): suffix array by prefix doubling with 64-bit positions, then the BWT
 * and the index.  ``d_text``: n uint32 symbols, T'[n-1] == 0 the unique
 * sentinel, n < 2^34.  ``keep_sa_text`` != 0 also keeps SA and T' on the
 * device for fm_locate / fm_extract_text.  The caller keeps ``d_text``. */
int fm_initialize_from_text_device(fm_index* h, const uint32_t* d_text, uint64_t n, int keep_sa_text,
                                   void* stream);

/* Adds locate / extract_text to an index built from a BWT alone
 * (fm_initialize_from_bwt_device) from ISA samples: d_isa[k] = the row of
 * text position 64 k, nisa = (n - 1) / 64 + 1 (sdsl's isa_sampling<> of a
 * csa_wt_int<>, i.e. what a reference .fmi holds next to its wavelet tree;
 * fm_index.cpp:196-209).  The SA samples are rebuilt by LF walks from them.
 * Every sample is checked (a row < n, and every 64-position walk must arrive at
 * its own block's sample), else -1 and nothing changes.  No reference
 * counterpart (the reference loads its .fmi through sdsl load_from_file). */
int fm_attach_isa_samples_device(fm_index* h, const uint64_t* d_isa, uint64_t nisa, void* stream);

/* The GPU suffix sorter on its own (current device, ``stream``): writes
 * BWT[j] = T'[SA[j] - 1 mod n] to ``d_bwt`` (n uint32, may be NULL) and the
 * suffix array to ``d_sa`` (n uint64, may be NULL). */
int fm_suffix_sort_device(const uint32_t* d_text, uint64_t n, uint32_t* d_bwt, uint64_t* d_sa,
                          void* stream);

/* The levelwise wavelet tree of sdsl's csa_wt_int<> (wt_int): level l =
 * the bits (MSB first) of the BWT stably sorted by its top l bits, packed
 * LSB-first into ceil(n/64) uint64 words per level, levels contiguous in
 * ``d_words`` (L * ceil(n/64) words).  For exporting sdsl-compatible level
 * vectors and for building the CPU baseline at full scale. */
int fm_wt_int_levels_device(const uint32_t* d_bwt, uint64_t n, uint32_t L, uint64_t* d_words,
                            void* stream);

/* ---- SWIG surface (host pointers, synchronous) ------------------------- */

/* FMIndex::size() -- fm_index.cpp:50-52: corpus tokens + 1 sentinel. */
int fm_size(const fm_index* h, uint64_t* out);

/* Number of distinct symbols in the BWT (sdsl wavelet_tree.sigma). */
int fm_sigma(const fm_index* h, uint64_t* out);

/* FMIndex::backward_search_step(symbol, low, high_inclusive) -- fm_index.cpp:67-97.
 * out[0..1] = half-open (low', high'), (0,0) when empty; high clamped to n-1. */
int fm_backward_search_step(fm_index* h, uint64_t symbol, uint64_t low, uint64_t high,
                            uint64_t out[2]);

/* FMIndex::backward_search_multi(query) -- fm_index.cpp:55-65: raw sdsl
 * backward_search chained from (0, n-1) with no early exit; out = (l, r+1). */
int fm_backward_search_multi(fm_index* h, const uint64_t* query, uint64_t len, uint64_t out[2]);

/* FMIndex::distinct(low, high) -- fm_index.cpp:99-117: ascending distinct
 * symbols of BWT[low, high).  Writes at most ``cap`` and the true count to *k. */
int fm_distinct(fm_index* h, uint64_t low, uint64_t high, uint64_t* syms, uint64_t cap,
                uint64_t* k);

/* FMIndex::distinct_count(low, high) -- fm_index.cpp:119-144: interleaved
 * [s0, c0, s1, c1, ...]; ``cap`` counts uint64 slots; *k = number of symbols. */
int fm_distinct_count(fm_index* h, uint64_t low, uint64_t high, uint64_t* out, uint64_t cap,
                      uint64_t* k);

/* FMIndex::distinct_count_multi(lows, highs) -- fm_index.cpp:146-166, one GPU
 * launch for all m ranges instead of one std::async per range.  Results of
 * range i are interleaved pairs at out[2*offsets[i] .. 2*offsets[i+1]);
 * ``offsets`` (m+1 entries) is written by the call; ``cap`` counts uint64
 * slots of ``out``.  Returns -2 (and offsets filled) if cap is too small. */
int fm_distinct_count_multi(fm_index* h, const uint64_t* lows, const uint64_t* highs,
                            uint64_t m, uint64_t* out, uint64_t cap, uint64_t* offsets);

/* Batched get_range (index.py:103-114) for host CSR patterns of token ids:
 * pattern i = tokens[offsets[i] .. offsets[i+1]); symbol = token + shift.
 * Starts at (0, n) (or (lo_in[i], hi_in[i]) when lo_in != NULL) and stops at
 * the first empty step with (0, 0). */
int fm_get_range_batch(fm_index* h, const int64_t* tokens, const int64_t* offsets, uint64_t m,
                       int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in,
                       uint64_t* lo_out, uint64_t* hi_out);

/* FMIndex::locate(row) -- fm_index.cpp:168-172: SA[row]; UINT64_MAX if row >= n.
 * From suffix-array samples (every 32nd text position, as sdsl csa_wt's
 * default): an LF walk of <= 31 steps on the GPU. */
int fm_locate(fm_index* h, uint64_t row, uint64_t* out);

/* FMIndex::extract_text(begin, end) -- fm_index.cpp:174-194 (LF walk from
 * isa[end-1], cyclic; isa from samples every 64 positions).  Writes
 * min(len, cap) symbols; *len = true length. */
int fm_extract_text(fm_index* h, uint64_t begin, uint64_t end, uint64_t* out, uint64_t cap,
                    uint64_t* len);

/* FMIndex::save(path) / load_FMIndex(path) -- fm_index.cpp:196-209.  Own
 * little-endian binary format (sdsl's serialization is not reproduced):
 * BWT + SA/ISA samples; everything else is rebuilt on load. */
int fm_save(fm_index* h, const char* path);
int fm_load(fm_index** out, const char* path, int device);
/* fm_load with the index built under `options` (NULL: the defaults). */
int fm_load_ex(fm_index** out, const char* path, int device, const fm_build_options* options);

/* ---- batched hot path (device pointers, stream-ordered) ---------------- */

/* One LF step per row for the incremental decode: state (lo[i], hi[i]) is a
 * half-open range with (0,0) meaning "empty"; symbol = tokens[i] + shift.
 * Equivalent to one iteration of index.py:109-112 (get_range's loop body),
 * i.e. backward_search_step(sym, lo, hi-1) with its (0,0) mapping; an empty
 * input state stays (0,0).  A row whose token is < reset_below restarts at
 * the full range (0, n) (a fresh sequence with an empty pattern); pass
 * INT64_MIN for plain get_range semantics.  lo_out/hi_out may alias lo/hi. */
int fm_lf_step_batch(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                     const uint64_t* d_lo, const uint64_t* d_hi,
                     uint64_t* d_lo_out, uint64_t* d_hi_out, uint64_t m, void* stream);

/* Device get_range for CSR patterns (same semantics as fm_get_range_batch). */
int fm_backward_search_batch(fm_index* h, const int64_t* d_tokens, const int64_t* d_offsets,
                             uint64_t m, int64_t shift, const uint64_t* d_lo_in,
                             const uint64_t* d_hi_in, uint64_t* d_lo_out, uint64_t* d_hi_out,
                             void* stream);

/* Allowed-next-token mask: mask[i*ld + t] = 1 iff symbol t+shift occurs in
 * BWT[lo[i], hi[i]) (t in [0, vocab)), else 0.  This is the boolean core of
 * every document_constrained_generation_* processor (the distinct list of
 * index.py:161-174 scattered into a vocab row).  ``packed`` != 0 writes a
 * bit mask instead (uint32 words, ld counts bytes and must be >= 4*ceil(vocab/32)). */
int fm_allowed_mask_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m,
                          uint8_t* d_mask, uint64_t ld, uint64_t vocab, int64_t shift,
                          int packed, void* stream);

/* Fused decode step, one launch: each row's LF step (as fm_lf_step_batch,
 * with restart for tokens < reset_below) from (d_lo_in, d_hi_in) into
 * (d_lo_out, d_hi_out), then the allowed mask of the new range.  The in and
 * out state buffers must not alias (callers ping-pong them); with vocab == 0
 * only the LF step runs and in-place update is allowed. */
int fm_decode_step_batch(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                         const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out,
                         uint64_t* d_hi_out, uint64_t m, uint8_t* d_mask, uint64_t ld,
                         uint64_t vocab, int packed, void* stream);

/* Device distinct_count for m ranges: ascending symbols + counts per row in
 * CSR slots d_cap_off[i] .. d_cap_off[i+1] (capacity, caller-computed as
 * min(hi-lo, sigma) prefix sums; total_cap = d_cap_off[m] known on the host);
 * the number written per row goes to d_k (UINT64_MAX = capacity overflow).
 * Uses the handle's shared workspace: refused (-1) on a capturing stream. */
int fm_distinct_count_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m,
                            const uint64_t* d_cap_off, uint64_t total_cap, uint64_t* d_syms,
                            uint64_t* d_counts, uint64_t* d_k, void* stream);

/* Batched locate (fm_index.cpp:168-172) for m device rows: d_out[i] =
 * SA[d_rows[i]] (UINT64_MAX for rows >= n), one LF walk per row, all rows in
 * parallel.  For get_doc_indices (index.py:123-129) over a whole range. */
int fm_locate_batch(fm_index* h, const uint64_t* d_rows, uint64_t m, uint64_t* d_out, void* stream);

/* Batched extract_text (fm_index.cpp:174-194): request i writes
 * d_out[d_off[i] .. d_off[i+1]) = the first d_off[i+1] - d_off[i] symbols of
 * extract_text(d_begin[i], d_end[i]) (the caller sizes d_off from the clamped
 * lengths min(end, n) - begin).  For get_doc (index.py:69-80) of many docs. */
int fm_extract_batch(fm_index* h, const uint64_t* d_begin, const uint64_t* d_end, const uint64_t* d_off,
                     uint64_t m, uint64_t* d_out, void* stream);

/* ---- fused logits-processor epilogue (no index needed) ------------------ */

/* Per-row parameters of fm_apply_boosts (32 bytes, packed as declared). */
typedef struct fm_row_params {
  float base;      /* mask value of every other token: 0.0 (soft) or -inf (hard) */
  float v_dist;    /* value of the allowed / distinct tokens */
  float v_uni;     /* value of all_unigrams not in the distinct set */
  float v_eos;     /* value of eos when FM_ROW_EOS is set (applied last) */
  uint32_t flags;  /* FM_ROW_* */
  int32_t reserved;
  int64_t special; /* the single distinct token when FM_ROW_SPECIAL is set */
} fm_row_params;

#define FM_ROW_BITS 1u     /* distinct set = bit row b of d_bits */
#define FM_ROW_UNIGRAM 2u  /* all_unigrams (d_unigram_bits) get v_uni */
#define FM_ROW_EOS 4u      /* token eos gets v_eos */
#define FM_ROW_SPECIAL 8u  /* token `special` is (also) in the distinct set */

/* out[b, t] = scores[b, t] + mask[b, t], the mask of the reference processors
 * (document_constrained_generation_causal_qwen.py:151-214 and the hard-mask
 * variants) assembled on the fly from the allowed-token bit rows of
 * fm_allowed_mask_batch(packed=1) and the per-row parameters, in the scores
 * dtype (0 = f32, 1 = bf16, 2 = f16) with torch's rounding.  Row values must
 * already be rounded to that dtype.  out may alias scores. */
int fm_apply_boosts(int dtype, const void* d_scores, void* d_out, uint64_t B, uint64_t V,
                    uint64_t ld_scores, uint64_t ld_out, const uint32_t* d_bits, uint64_t ld_bits,
                    const uint32_t* d_unigram_bits, const fm_row_params* d_rows, int64_t eos,
                    void* stream);

/* ---- doc-range sharding (no index needed) ------------------- */

/* The exchange step of a sharded decode: OR of the bit-packed allowed rows of
 * ``nparts`` shards (block p = d_parts + p * part_stride words, B rows of
 * words_per_row uint32, fm_allowed_mask_batch(packed=1)'s bit order -- what an
 * RCCL all_gather of every rank's decode-step output holds).  unpack != 0
 * writes the uint8 [B, vocab] 0/1 mask (ld_out bytes per row); 0 the ORed
 * words (ld_out bytes per row, a multiple of 4).  Stream-ordered. */
int fm_or_bits(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t words_per_row,
               uint64_t vocab, void* d_out, uint64_t ld_out, int unpack, void* stream);

/* The sparse exchange (replaces shipping every row's bitmap): a rank packs,
 * per row of its post-step state (d_lo, d_hi) on its shard, either the BWT
 * slice [lo, hi) (when hi - lo < W = ceil(vocab / 32): smaller than the
 * bitmap) or the row's bitmap from d_bits (its fm_decode_step_batch(packed=1)
 * output, ldw words per row) into d_payload (cap_words uint32; word 0 = the
 * words used, a multiple of 4: an all_gather needs only the largest rank's
 * prefix).  fm_shard_or_rows ORs the payloads of nparts ranks (part p at
 * d_parts + p * part_stride words) into the uint8 [B, vocab] mask (unpack != 0)
 * or the packed words -- bit for bit what fm_or_bits gives for the ranks'
 * bitmaps (a BWT symbol s is token s - shift, kept when in [0, vocab)).
 * Layout: csrc/shard.hip.  Replaces the dense OR-exchange SURVEY §8e
 * describes (all_gather of packed [B, V/32] rows). */
int fm_shard_payload_capacity(uint64_t B, uint64_t vocab, uint64_t* words);
/* The decode step (fm_decode_step_batch's LF step, packed) writing the exchange
 * payload itself, with FIXED row slots (row b at H + b * round4(W) words, the
 * capacity fm_shard_payload_capacity gives): a row whose new range is narrower
 * than W and streamed whole gets its BWT slice, every other row its bitmap; no
 * pack pass.  For payloads read in place (fm_shard_or_rows_peers), whose wire
 * cost is what the reader reads, not the capacity; an all_gather would ship the
 * whole capacity (use fm_shard_pack there).  vocab <= 262144; d_payload 16-B
 * aligned, cap_words >= fm_shard_payload_capacity(m, vocab). */
/* The state may be updated in place (d_lo_out == d_lo_in, d_hi_out == d_hi_in), so a captured step
 * replays for every step.  With d_step != NULL (the flag barrier's device step counter) the kernel
 * writes d_payload when *d_step is even and d_payload_alt when it is odd -- the peer exchange's
 * double buffer picked on the device, in step with fm_shard_or_rows_peers_wait; NULL: d_payload. */
int fm_decode_step_payload(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                           const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out, uint64_t* d_hi_out,
                           uint64_t m, uint32_t* d_payload, uint64_t cap_words, uint64_t vocab,
                           uint32_t* d_payload_alt, const uint32_t* d_step, void* stream);
/* The same step with the flag barrier's signal fused in (fm_peer_signal without its own launch):
 * every workgroup, once its payload stores are acknowledged, arrives on d_done (288 uint32 zeroed once:
 * nine counters 32 words apart -- one per residue of the workgroup index mod 8, then their join --
 * reset by the kernel itself); the last one does fm_peer_signal's work -- a system-scope
 * release, step = *d_step + 1 stored into every rank's flag word for this rank (d_flag_ptrs[world]),
 * *d_step = step.  A flag-barrier step is then two launches (this, fm_shard_or_rows_peers_wait). */
int fm_decode_step_payload_signal(fm_index* h, const int64_t* d_tokens, int64_t shift, int64_t reset_below,
                                  const uint64_t* d_lo_in, const uint64_t* d_hi_in, uint64_t* d_lo_out,
                                  uint64_t* d_hi_out, uint64_t m, uint32_t* d_payload, uint64_t cap_words,
                                  uint64_t vocab, uint32_t* d_payload_alt, uint32_t* d_step,
                                  const uint64_t* d_flag_ptrs, uint64_t world, uint32_t* d_done, void* stream);
/* One flag-barrier step in one call (the per-step host work of ShardedDecoder's flag path: no
 * Python between the launches): fm_decode_step_payload_signal on the state in place, then
 * fm_shard_or_rows_peers_wait into d_out; with sync != 0 the stream is then synchronised and the
 * host-mapped error word read, and a step whose barrier timed out returns 1 (its output is not
 * exact: exact or absent).  The step's buffers, fixed across steps, travel in one struct. */
typedef struct fm_peer_step {
  uint64_t* d_lo;              /* the rows' state, updated in place */
  uint64_t* d_hi;
  uint64_t m;
  uint32_t* d_payload;         /* the double-buffered payload (the counter's parity picks) */
  uint32_t* d_payload_alt;
  uint64_t cap_words;
  uint32_t* d_step;            /* the device step counter */
  const uint64_t* d_flag_ptrs; /* this rank's word in every rank's flag array */
  uint64_t world;
  uint32_t* d_done;            /* 288 words, zero (the fused signal's arrival counts) */
  const uint64_t* d_part_ptrs; /* [2, nparts]: every rank's two payload buffers */
  uint64_t nparts;
  const uint32_t* d_flags;     /* this rank's flag array */
  uint32_t spins;
  uint32_t* err;               /* host-mapped error word (fm_host_mapped_alloc) */
  void* d_out;
  uint64_t ld_out;
  int32_t unpack;
  uint64_t vocab;
  int64_t shift;
  int64_t reset_below;
} fm_peer_step;
int fm_peer_flags_step(fm_index* h, const fm_peer_step* p, const int64_t* d_tokens, int sync, void* stream);
int fm_shard_pack(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t B, const uint32_t* d_bits,
                  uint64_t ldw, uint64_t vocab, uint32_t* d_payload, uint64_t cap_words, void* stream);
int fm_shard_or_rows(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t vocab,
                     int64_t shift, void* d_out, uint64_t ld_out, int unpack, void* stream);
/* The same two carrying a doc-sharded processor call's per-row facts in the
 * payload (no collective for them; SURVEY §8e: "emptiness flags and
 * count([last]) > 0 are also exact via OR"): fm_shard_pack_facts stores d_facts
 * (int32 [3, B]: count([last]) > 0, range non-empty, distinct non-empty, as
 * fm_processor_shard_prep writes them) in the payload's facts area;
 * fm_shard_or_rows_facts writes their OR over the parts to d_facts_out (int32
 * [3, B], 0/1) -- what fm_processor_shard_finish takes for the facts summed over
 * the ranks.  fm_shard_pack (no facts) leaves the area zero. */
int fm_shard_pack_facts(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t B, const uint32_t* d_bits,
                        uint64_t ldw, uint64_t vocab, const int32_t* d_facts, uint32_t* d_payload, uint64_t cap_words,
                        void* stream);
int fm_shard_or_rows_facts(const uint32_t* d_parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t vocab,
                           int64_t shift, void* d_out, uint64_t ld_out, int unpack, int32_t* d_facts_out,
                           void* stream);

/* The peer exchange (no host read, no gather): every rank packs into one of
 * two payload buffers of fm_shard_payload_capacity words (double-buffered by
 * step parity), whose IPC handles the ranks swapped once (fm_ipc_handle /
 * fm_ipc_open: hipIpc*, the peer mapping over xGMI); after a stream-ordered
 * barrier (any collective every rank issues after its pack, e.g. the
 * processors' facts all_reduce), fm_shard_or_rows_peers reads the nparts
 * payloads in place through d_part_ptrs (a device array of nparts addresses,
 * each payload cap_words words), with system-scope loads, and ORs them as
 * fm_shard_or_rows does.  fm_ipc_handle returns the allocation's handle
 * (FM_IPC_HANDLE_BYTES) and d_ptr's offset in it; fm_ipc_open maps a peer's
 * allocation (its base: add the offset); fm_ipc_close unmaps it.  Not in the
 * reference (its OR-exchange is an all_gather). */
#define FM_IPC_HANDLE_BYTES 64
int fm_shard_or_rows_peers(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                           uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack, void* stream);
/* The flag barrier instead of a collective: each rank owns a uint32 flag word per
 * rank (d_flags[world], zeroed, IPC-shared) and a uint32 step counter d_step
 * (device, zeroed).  fm_peer_signal: step = *d_step + 1 (mod 2^32); a
 * system-scope release (the payload the previous kernel on the stream wrote is
 * visible before any flag says so), step stored into every rank's word for this
 * rank (d_flag_ptrs[world]: the peers' word addresses, mapped; system-scope
 * vector stores), *d_step = step -- issue it after the kernel that wrote this
 * rank's payload; world = 0 advances the counter and posts nothing.
 * fm_shard_or_rows_peers_wait: step = *d_step; the payloads are
 * d_part_ptrs[((step - 1) & 1) * nparts ..] (d_part_ptrs holds buffer 0's
 * nparts addresses, then buffer 1's); waits until every (int32)(d_flags[p] -
 * step) >= 0 (system-scope polls, at most `spins`, 0 = 2^20 ~ 0.1-1 s), then a
 * system-scope acquire, then ORs as fm_shard_or_rows_peers.  On timeout
 * *err = step (a system-scope store: err may be fm_host_mapped_alloc memory,
 * read by the host without a synchronisation) and the pass goes on, so the
 * grid drains -- its output is then NOT exact and the caller must raise.
 * The step number lives on the device, so decode + signal + OR captured once
 * into a graph replay for every step. */
int fm_peer_signal(const uint64_t* d_flag_ptrs, uint64_t world, uint32_t* d_step, void* stream);
/* The persistent LF sweep (fm_tuning lf_work = 4, fm_lf_step_batch from lf_sweep_min rows on a stream
 * that is not capturing): after a synchronisation with its last launch, *err != 0 if a launch gave up
 * a wait (its rows are then not all stepped).  Its grid is the resident wave count and a drainer may
 * wait on another wave's heads, so a launch beside other work that keeps its waves off the chip can
 * end this way; the in-wave sweep (lf_work -1, the default) has no such wait. */
int fm_lf_persist_status(fm_index* h, uint32_t* err);
int fm_shard_or_rows_peers_wait(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                                uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack,
                                const uint32_t* d_flags, const uint32_t* d_step, uint32_t spins, uint32_t* err,
                                void* stream);
/* Either peer pass (d_flags NULL: fm_shard_or_rows_peers, else
 * fm_shard_or_rows_peers_wait) with the facts' OR written to d_facts_out, as
 * fm_shard_or_rows_facts: a sharded processor call over the flag barrier holds
 * no collective at all. */
int fm_shard_or_rows_peers_facts(const uint64_t* d_part_ptrs, uint64_t nparts, uint64_t cap_words, uint64_t B,
                                 uint64_t vocab, int64_t shift, void* d_out, uint64_t ld_out, int unpack,
                                 const uint32_t* d_flags, const uint32_t* d_step, uint32_t spins, uint32_t* err,
                                 int32_t* d_facts_out, void* stream);
/* Coherent host memory mapped for the device (hipHostMalloc mapped | coherent),
 * zeroed: kernels store into it, the host reads it without a copy (the flag
 * barrier's error word). */
int fm_host_mapped_alloc(uint64_t bytes, void** out);
int fm_host_mapped_free(void* p);
int fm_ipc_handle(const void* d_ptr, uint8_t* handle, uint64_t* offset);
int fm_ipc_open(const uint8_t* handle, void** d_base);
int fm_ipc_close(void* d_base);

/* ---- logits-processor step on the device --------------------------------- */

/* The per-row bookkeeping of the soft processors' _process
 * (document_constrained_generation_causal_qwen.py:101-214,
 * document_constrained_generation_causal.py:74-180), one wave per row. */
typedef struct fm_prep_config {
  int64_t marker[8];       /* remove_end_marker's marker, marker_len tokens (causal_qwen.py:42,44-56) */
  int64_t think[2];        /* finished_thinking's pair (causal_qwen.py:76) */
  int64_t sys[4];          /* remove_system_tokens' prefix (causal_qwen.py:60) */
  int64_t eos, pad, stop_at_count, min_new_tokens, forced_bos, shift;
  int32_t marker_len;      /* 1..8 */
  int32_t num_beams;       /* rows = batch x num_beams, beams of one batch item adjacent */
  uint32_t flags;          /* FM_PREP_* */
  float base;              /* mask value of untouched tokens (0.0 for the soft processors) */
  float v_uni_full;        /* BOOST rounded to the scores dtype */
  float v_uni_half;        /* BOOST / 2 rounded */
  float v_forced;          /* BOOST rounded (forced bos) */
  int32_t skip;            /* FM_PREP_HARD: leading tokens that are not pattern (seq: the decoder start) */
} fm_prep_config;

#define FM_PREP_THINK 1u       /* think gating + system-token removal (Qwen) */
#define FM_PREP_SKIP_FIRST 2u  /* forced_bos_token_id set: strip the first generated token (causal.py:80-85) */
#define FM_PREP_EOS 4u         /* always_allow_eos */
#define FM_PREP_EOS_ALL 8u     /* the eos boost on every row, no min_new_tokens gate (causal.py:173-178) */
#define FM_PREP_UNI_HALF 16u   /* BOOST / 2 for the other unigrams even when distinct is empty (causal.py:171) */
#define FM_PREP_HARD 32u       /* the hard-mask variants (vllm.py:46-137, seq.py:35-123): no end marker, the
                                  pattern is every token from `skip` on, no trailing n-gram rule, and
                                  stop_at_count tests the count of the pattern without its last token */

#define FM_PREP_BAD_MARKER 1u  /* status: a row without exactly one end marker */
#define FM_PREP_BAD_POW 2u     /* status: a boost BOOST * lrf^k outside the table (Python float overflow) */

/* One processor step on the device, for B rows of d_ids (int64 [B, L], ld_ids
 * elements per row): end marker, think gating, system tokens, the trailing
 * n-gram rule (count of the last token), the eos / pad / stop_at_count rules,
 * and the pattern range -- ONE LF step from the previous call's range of the
 * row whose pattern this one extends (d_prev_ids / d_prev_state, rows of the
 * same beam group, compared token by token), else a full search of
 * force_decoding_from + sent (index.py:103-114).  Writes the epilogue's row
 * parameters (d_rows), the range of every row whose distinct set is the
 * mask's (d_mask_lo / d_mask_hi, (0, 0) otherwise) and this call's state
 * d_state = int64 [4][B] (pattern start in the row, length or -1, lo, hi).
 * d_pow[k] = BOOST * lrf^k rounded to the scores dtype (NaN: not a finite
 * Python float).  d_status (4 uint32, written by the call): [0] FM_PREP_BAD_*
 * bits, [1] / [2] min / max marker end over the rows (they must agree, as
 * the reference's torch.stack requires).  Stream-ordered; no allocation. */
int fm_processor_step(fm_index* h, const fm_prep_config* cfg, const int64_t* d_ids, uint64_t B, uint64_t L,
                      uint64_t ld_ids, const int64_t* d_fdf, uint64_t fdf_len, const float* d_pow, uint64_t pow_len,
                      const int64_t* d_prev_ids, uint64_t prev_ld, uint64_t prev_B, const int64_t* d_prev_state,
                      fm_row_params* d_rows, uint64_t* d_mask_lo, uint64_t* d_mask_hi, int64_t* d_state,
                      uint32_t* d_status, void* stream);

/* One whole processor call (the three launches of the device path plus the
 * hand-offs), so the host makes one call per decode step:
 *   fm_processor_step (which also copies this call's ids to ids_copy, the next
 *   call's prev_ids, optional) -> fm_allowed_mask_batch(packed) of
 *   (mask_lo, mask_hi) into bits -> fm_apply_boosts(scores -> out).  The status
 *   is copied to status_host (pinned, optional) right after fm_processor_step,
 *   and status_event (a hipEvent_t, optional) is recorded behind that copy: the
 *   caller waits on the event -- the row bookkeeping only -- before reading
 *   status_host, while the mask and the epilogue still run.  With neither, the
 *   status is not even initialised (a hard-mask call's status is fixed by its
 *   inputs: no end marker, zero boosts), so the call needs no host wait at
 *   all.  Stream-ordered.  Replaces the per-call work of
 *   document_constrained_generation_causal_qwen.py:101-214 / causal.py:62-180. */
typedef struct fm_processor_args {
  const int64_t* ids;          /* [B][ld] input_ids */
  uint64_t B, L, ld;
  const int64_t* fdf;          /* force_decoding_from tokens */
  uint64_t fdf_len;
  const float* pow_tab;        /* boost table (fm_processor_step) */
  uint64_t pow_len;
  const int64_t* prev_ids;     /* previous call's ids [prev_B][prev_ld], or null */
  uint64_t prev_ld, prev_B;
  const int64_t* prev_state;   /* previous call's state [4][prev_B] */
  fm_row_params* rows;         /* [B] out */
  uint64_t* mask_lo;           /* [B] out */
  uint64_t* mask_hi;           /* [B] out */
  int64_t* state;              /* [4][B] out */
  uint32_t* status;            /* [4] device */
  uint32_t* bits;              /* [B][bits_ld] packed allowed bits (scratch) */
  uint64_t bits_ld;            /* uint32 words per row, >= ceil(V/32) */
  int32_t dtype;               /* of scores / out: 0 = f32, 1 = bf16, 2 = f16 */
  int32_t reserved;
  const void* scores;          /* [B][ld_scores] */
  void* out;                   /* [B][ld_out] */
  uint64_t V, ld_scores, ld_out;
  const uint32_t* unigram_bits;
  int64_t eos;
  int64_t* ids_copy;           /* [B][copy_ld] or null; must not overlap prev_ids or ids (rejected) */
  uint64_t copy_ld;
  uint32_t* status_host;       /* pinned [4] or null */
  void* status_event;          /* hipEvent_t recorded after the status copy, or null */
} fm_processor_args;

int fm_processor_call(fm_index* h, const fm_prep_config* cfg, const fm_processor_args* args, void* stream);

/* A processor call over a doc-range SHARD of the corpus (masks,
 * emptiness and count([last]) > 0 are exact under an OR over the shards), in
 * two phases around the caller's exchange:
 *   fm_processor_shard_prep (every rank, on its shard): fm_processor_step with
 *   the index-dependent decisions recorded instead of taken -- d_facts int32
 *   [3][B] = this shard's (count([last]) > 0, pattern range non-empty, distinct
 *   set non-empty) as 0/1, d_rowcase [B] = the row's case (0: decided without
 *   the index, 1: eos / pad last token, 2: pattern searched) | pattern length
 *   << 2 -- then the shard's packed allowed bits of every searched row into
 *   args->bits.  args->status [3] receives the longest searched pattern
 *   (force_decoding_from included), to be checked against the shards' halo.
 *   The caller sums d_facts over the ranks (all_reduce SUM) and ORs the bits
 *   (fm_or_bits / the sparse exchange).
 *   fm_processor_shard_finish: decides those rows from the sums exactly as
 *   fm_processor_step decides them on one index, copies the status (+ event,
 *   as fm_processor_call), and runs the epilogue with the ORed bits (d_bits,
 *   bits_ld words per row).
 * stop_at_count must be 0 (a shard's counts include its halo's duplicates;
 * every reference call site passes 0).  No index is needed for the finish. */
#define FM_PREP_BAD_HALO 4u    /* status (host side): a pattern longer than the shards' halo allows */
int fm_processor_shard_prep(fm_index* h, const fm_prep_config* cfg, const fm_processor_args* args, int32_t* d_facts,
                            uint32_t* d_rowcase, void* stream);
int fm_processor_shard_finish(const fm_prep_config* cfg, const fm_processor_args* args, const int32_t* d_facts_sum,
                              const uint32_t* d_rowcase, const uint32_t* d_bits, uint64_t bits_ld, void* stream);

/* ---- introspection (bench / roofline accounting) ----------------------- */

/* Digit levels of the wavelet matrix (the 2-level one: one dependent rank
 * round trip each per LF step) and its bytes, bytes of the plain BWT (0 once
 * E holds the symbols) and of the bitmaps, the aligned bitmap block. */
int fm_stats(const fm_index* h, uint64_t* levels, uint64_t* wm_bytes, uint64_t* bwt_bytes,
             uint64_t* bitmap_bytes, uint64_t* bitmap_block);

/* Bytes of the LF path's 2-level wavelet matrix and its level count, and the
 * range-bitmap cache: cached ranges (every SA range reachable from the root
 * with width >= cache_min), their bytes, and cache_min (0 = no cache). */
int fm_stats_ex(const fm_index* h, uint64_t* w2_levels, uint64_t* w2_bytes, uint64_t* cache_nodes,
                uint64_t* cache_bytes, uint64_t* cache_min);

/* Transition table of the cached ranges (cached parent, symbol) -> child range:
 * entries inserted, entries left out (both buckets full; those steps take the
 * wavelet-matrix descent) and bytes in HBM. */
int fm_stats_trans(const fm_index* h, uint64_t* entries, uint64_t* dropped, uint64_t* bytes);

/* 1 when the transition table holds every child of every cached parent (transitions = 2,
 * trans_min = 1, nothing skipped): a probe that finds no key beside a free slot then proves
 * the symbol absent and the LF step ends after the probe; 0 otherwise (or with
 * FMIDX_PROBE_COMPLETE=0 at build time). */
int fm_stats_trans_complete(const fm_index* h, uint32_t* complete);

/* Device memory of the index: the E array, the SA/ISA samples and the total
 * of every device structure (bytes). */
int fm_stats_mem(const fm_index* h, uint64_t* e_bytes, uint64_t* sample_bytes, uint64_t* total_bytes);

/* For m device ranges, out[i] = 1 if [lo[i], hi[i]) has a cached bitmap
 * (accounting / tests; stream-ordered). */
int fm_cache_lookup_batch(fm_index* h, const uint64_t* d_lo, const uint64_t* d_hi, uint64_t m, uint8_t* d_out,
                          void* stream);

/* HBM gather probe (bench roofline of the rank/LF path); no
 * index needed, current device.  ``chase`` selects the access pattern over
 * d_buf[0, bytes), ``threads`` threads each issuing ``loads`` loads:
 *   0: every thread its own random 64-B line (4 x 16 B) -- per-lane lines;
 *   1: ``threads`` chains each follow ``loads`` dependent hops (next line =
 *      the uint64 at the start of the current line mod the line count);
 *   2: 4 lanes share a random 64-B line, 16 B each (lane-cooperative);
 *   3: 8 lanes share a random 128-B line, 16 B each;
 *   4: every thread its own random 8-B word.
 * Line counts are powers of two (the largest that fits).  d_sink: >= 1024
 * uint64 (practically never written). */
int fm_probe_gather(const void* d_buf, uint64_t bytes, int chase, uint64_t loads, uint32_t threads,
                    uint64_t* d_sink, void* stream);

/* Device pointer to the plain BWT (uint32[n]) for samplers / bench traces.
 * When the index keeps no plain BWT (E holds its symbols: the default), the
 * first call MATERIALISES a copy (n * 4 bytes of HBM, held by the handle and
 * not counted in fm_stats_mem's total: see fm_stats_views) -- release it with
 * fm_release_bwt_view once done (it synchronises the device). */
int fm_device_bwt(const fm_index* h, const uint32_t** out);
int fm_release_bwt_view(fm_index* h);
/* Bytes the handle holds outside its query structures: the BWT copy
 * fm_device_bwt materialised (0 when none). */
int fm_stats_views(const fm_index* h, uint64_t* bwt_view_bytes);

/* Device pointer and byte size of one index structure, for the bench's
 * gather ceilings over the index's own allocations: which = 0 plain BWT,
 * 1 E array, 2 transition table, 3 range-bitmap cache, 4 first level of the
 * 2-level wavelet matrix.  *out = NULL, *bytes = 0 when the structure is not
 * built.  (Measurement only; no reference counterpart.) */
int fm_device_struct(const fm_index* h, int which, const void** out, uint64_t* bytes);

/* Synchronise the handle's device (hipDeviceSynchronize on its device). */
int fm_synchronize(fm_index* h);

/* Restores the launch tuning to the library defaults with the FMIDX_TUNING
 * overrides (re-read) on top.  Call it while no launch is being issued.  No
 * reference counterpart. */
int fm_reload_tuning(void);

#ifdef __cplusplus
}
#endif

#endif /* FMIDX_H_ */
