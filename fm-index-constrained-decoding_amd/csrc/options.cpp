// options.cpp -- index-structure options and launch tuning (include/fmidx.h:
// fm_build_options, fm_tuning).  Values come from the API; the environment
// holds at most two override strings, FMIDX_BUILD_OPTIONS and FMIDX_TUNING
// ("key=value,key=value"), for measurement runs that cannot change code.
#include "fmidx_internal.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace fmidx {

namespace {

// "key=value[,| ]key=value..." -> set(key, value) for each; false on a malformed pair or a key
// `set` rejects
template <typename F>
bool parse_kv(const char* spec, F set) {
  std::string s(spec ? spec : "");
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && (s[i] == ',' || s[i] == ' ' || s[i] == ';')) ++i;
    if (i >= s.size()) break;
    size_t j = i;
    while (j < s.size() && s[j] != ',' && s[j] != ' ' && s[j] != ';') ++j;
    const std::string kv = s.substr(i, j - i);
    const size_t eq = kv.find('=');
    if (eq == std::string::npos || eq == 0 || eq + 1 >= kv.size()) return false;
    char* end = nullptr;
    const std::string val = kv.substr(eq + 1);
    const long long x = std::strtoll(val.c_str(), &end, 0);
    if (!end || *end) return false;
    if (!set(kv.substr(0, eq), x)) return false;
    i = j;
  }
  return true;
}

bool set_build(BuildOpts& o, const std::string& k, long long x) {
  if (k == "profile") o = build_profile((int)x);
  else if (k == "transitions" || k == "trans") o.transitions = (int32_t)x;
  else if (k == "lf_e") o.lf_e = (int32_t)x;
  else if (k == "lf_e2") o.lf_e2 = (int32_t)x;
  else if (k == "probe_first") o.probe_first = (int32_t)x;
  else if (k == "keep_bwt") o.keep_bwt = (int32_t)x;
  else if (k == "follow_bitmaps") o.follow_bitmaps = (int32_t)x;
  else if (k == "bm_log2") o.bm_log2 = (int32_t)x;
  else if (k == "trans_min") o.trans_min = (int32_t)x;
  else if (k == "cache_min") o.cache_min = (uint64_t)x;
  else if (k == "cache_mb") o.cache_mb = (uint64_t)x;
  else if (k == "trans_mb") o.trans_mb = (uint64_t)x;
  else if (k == "gpu_sort_min") o.gpu_sort_min = (uint64_t)x;
  else return false;
  return true;
}

bool set_tuning_kv(Tuning& t, const std::string& k, long long x) {
  if (k == "lf_group") t.lf_group = (uint32_t)x;
  else if (k == "search_group") t.search_group = (uint32_t)x;
  else if (k == "dec_threads") t.dec_threads = (uint32_t)x;
  else if (k == "mask_slices") t.mask_slices = (uint32_t)x;
  else if (k == "lf_group_min") t.lf_group_min = (uint64_t)x;
  else if (k == "lf_work") t.lf_work = (int32_t)x;
  else if (k == "lf_gprobe") t.lf_gprobe = (int32_t)x;
  else if (k == "lf_quad") t.lf_quad = (int32_t)x;
  else if (k == "lf_split") t.lf_split = (int32_t)x;
  else if (k == "search_p8") t.search_p8 = (int32_t)x;
  else if (k == "lf_sweep_min") t.lf_sweep_min = (uint64_t)x;
  else if (k == "sa_chunk") t.sa_chunk = (uint64_t)x;
  else return false;
  return true;
}

bool valid_group(uint32_t g) { return g == 1 || g == 2 || g == 4 || g == 8 || g == 16 || g == 64; }

bool check_tuning(const Tuning& t) {
  if (!valid_group(t.lf_group) || !valid_group(t.search_group)) {
    set_error("tuning: lanes per row must be 1, 2, 4, 8, 16 or 64");
    return false;
  }
  if (t.dec_threads && t.dec_threads != 256 && t.dec_threads != 512 && t.dec_threads != 1024) {
    set_error("tuning: dec_threads must be 0, 256, 512 or 1024");
    return false;
  }
  if (t.lf_work < -1 || t.lf_work > 4 || t.lf_work == 3) {
    set_error("tuning: lf_work must be -1 (by row count), 0, 1, 2 or 4");
    return false;
  }
  if (t.sa_chunk < 1024) {
    set_error("tuning: sa_chunk below 1024 rows");
    return false;
  }
  return true;
}

std::mutex g_tuning_mu;

Tuning& tuning_slot() {
  static Tuning t = [] {
    Tuning d;
    const char* e = std::getenv("FMIDX_TUNING");
    if (e && *e) {
      Tuning o = d;
      if (parse_kv(e, [&](const std::string& k, long long x) { return set_tuning_kv(o, k, x); }) && check_tuning(o))
        d = o;
      else
        std::fprintf(stderr, "[fmidx] FMIDX_TUNING=%s ignored (malformed or out of range)\n", e);
    }
    return d;
  }();
  return t;
}

}  // namespace

BuildOpts build_profile(int profile) {
  BuildOpts o;
  o.profile = profile;
  if (profile == 1) {   // compact: transitions to cached children only, no E array, probe with the descent
    o.transitions = 1;
    o.lf_e = 0;
    o.probe_first = 0;
  }
  return o;
}

int apply_build_overrides(BuildOpts& o) {
  const char* e = std::getenv("FMIDX_BUILD_OPTIONS");
  if (!e || !*e) return 0;
  BuildOpts x = o;
  if (!parse_kv(e, [&](const std::string& k, long long v) { return set_build(x, k, v); })) {
    set_error("FMIDX_BUILD_OPTIONS=%s: expected key=value pairs of fm_build_options fields", e);
    return -1;
  }
  o = x;
  return 0;
}

const Tuning& tuning() { return tuning_slot(); }

int set_tuning(const Tuning& t) {
  Tuning x = t;
  const char* e = std::getenv("FMIDX_TUNING");
  if (e && *e && !parse_kv(e, [&](const std::string& k, long long v) { return set_tuning_kv(x, k, v); })) {
    set_error("FMIDX_TUNING=%s: expected key=value pairs of fm_tuning fields", e);
    return -1;
  }
  if (!check_tuning(x)) return -1;
  std::lock_guard<std::mutex> lk(g_tuning_mu);
  tuning_slot() = x;
  return 0;
}

}  // namespace fmidx
