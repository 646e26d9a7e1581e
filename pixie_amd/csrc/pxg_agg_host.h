// Host-side state of one aggregation (pxg_agg).
#pragma once

#include <vector>

#include "pxg_agg.h"
#include "pxg_sort.h"

namespace pxg {

struct HcExport;  // pxg_hc.hip

struct AggResult {
  int64_t n_groups = 0;
  bool ready = false;
  // device outputs (dense by group)
  DevBuf key_fixed[kMaxKeys];   // 8 or 16 B per group
  DevBuf key_offsets[kMaxKeys]; // STRING: int32 offsets (n+1)
  DevBuf key_data[kMaxKeys];
  int64_t key_data_len[kMaxKeys] = {0};
  DevBuf uda_out[kMaxUdas];     // 8 B per group (QUANTILES: 7 doubles per group)
  DevBuf states;                // emit_states: state_rec bytes per group (Serialize layout)
  DevBuf lanes;                 // pxg_agg_quantile_lanes scratch
  // Forget the result; device buffers stay allocated for the next finalize.
  void Clear() {
    n_groups = 0;
    ready = false;
    for (auto& l : key_data_len) l = 0;
  }
};

struct Agg {
  Ctx* ctx = nullptr;
  int32_t n_keys = 0, n_udas = 0, n_vals = 0;
  bool windowed = false;
  bool has_filter = false;
  bool emit_states = false;  // partial_agg && !finalize_results: result = groups + states
  int32_t state_rec = 0;
  // Keys for the consume fast path (AggConsumeFastKernel<fast_nk>); 0 = generic kernel.
  int32_t fast_nk = 0;
  std::vector<int32_t> uda_kind, uda_arg_type, uda_val, uda_out_type;
  std::vector<int64_t> uda_init;
  std::vector<int32_t> uda_has_init;
  std::vector<int32_t> key_types;
  std::vector<int32_t> val_type;
  // Programs reference input columns by index/type; checked against each consumed table.
  std::vector<std::pair<int32_t, int32_t>> col_refs;  // (col, type)

  AggPlanDev hplan;
  DevBuf d_plan;
  DevBuf d_pool;

  // Multi-GPU exchange of partial states (pxg_xchg.hip).  hplan_x: the plan with
  // every non-quantile UDA's Serialize() state laid out per group (GroupCombine writes them in
  // export mode); x_ok: the plan can exchange states (no windowing / partial-emit / MINSUM /
  // MEAN_MERGE, all quantile UDAs on one value stream x_qval, -1: none).
  AggPlanDev hplan_x;
  DevBuf d_plan_x;
  bool x_ok = false;
  int32_t x_qval = -1;
  bool export_x = false;       // finalize runs for an export: states + centroid lists, below
  bool x_check_pending = false;  // an export finalize left its checks to CheckExportFinalize
  uint32_t x_check_groups = 0;   // ... and the group count the device must agree with
  const uint64_t* x_vals = nullptr;  // after an export finalize: the grouped quantile stream
  uint32_t x_nbig = 0;               // ... and its big groups (ws.big / ws.xcent / ws.xcnt)
  // Owner side: imported states merged per slot (macc: macc_words u64 per slot at macc_off[u],
  // plus a flags word) and quantile items staged with a weight stream (st_wt: part << 48 |
  // weight, 0 = raw value).  merged: this run holds imported states (consume refused).
  bool merged = false;
  DevBuf macc, st_wt;
  uint32_t macc_cap = 0;
  int32_t macc_words = 0;
  int32_t macc_off[kMaxUdas] = {0};
  int32_t x_parts_seen = 0;   // part index of the next imported part (weights carry it)
  int32_t EnsureMacc();
  int32_t FinalizeMerged();
  const uint64_t* x_wts = nullptr;  // after a merged finalize: the grouped item weights

  // Global open-addressing table.
  DevBuf slots;
  // Probe records (pxg_agg.h kRecWords per slot), allocated with the table when the plan
  // qualifies (rec_ok: consume fast path, all-STRING keys, <= kRecMaxKeys); rec_dirty: written
  // since the last clear.
  DevBuf prec;
  bool rec_ok = false, rec_dirty = false;
  uint32_t rec_cap = 0;
  int32_t EnsureRecords();
  int32_t RebuildRecords();
  uint32_t cap = 0;
  uint32_t min_cap = 1024;  // the capacity the creation hint asked for (reset never shrinks below)
  DevBuf counters;  // u32 [0] groups in the table (fill guard) [2] deferred rows ; u64 @16 staging cursor;
                    // u32 @32 import inserts, @36 import error flags
  DevBuf deferred[2], deferred_pos[2];
  DevBuf d_ranges;
  std::vector<uint8_t> last_ranges;  // host copy of what d_ranges holds
  DevBuf arena;
  uint64_t arena_words = 0;  // used (host mirror after publish)
  uint32_t last_big_sort_groups = 0;  // pxg_agg_stats.big_sort_groups
  uint64_t inserted = 0;     // host mirror
  uint64_t last_groups = 0;  // groups of the last run with any (table sizing across resets)

  // Staging (one record per selected row).
  DevBuf st_slot;
  DevBuf st_val[kMaxVals];
  uint64_t st_cap = 0;
  uint64_t st_n = 0;  // host mirror of the cursor

  // High-cardinality mode (pxg_hc.hip): chosen at the first consume after create / reset when
  // the plan qualifies (hc_ok) and the hint or the last run says >= kHcMinGroups groups.  Rows
  // are staged as partition records instead of probing the global table; finalize partitions
  // them by hash and aggregates each partition in one workgroup's LDS table.
  bool hc_ok = false;      // plan-level eligibility (pxg_agg_create)
  bool hc_active = false;  // this run stages partition records
  int64_t hint_groups = 0;
  HcStageDev hc_layout{};  // stride / key words (pointers filled per launch)
  DevBuf hc_rec, hc_key;
  DevBuf hc_maxlen;                       // u32 [kMaxKeys], device
  uint32_t hc_maxlen_h[kMaxKeys] = {0};   // host mirror (read with the publish counters)
  uint64_t hc_cap = 0;
  uint64_t hc_n = 0;  // host mirror of the record cursor (counters @48)
  int32_t last_hc_pbits = 0;  // partition bits of the last finalize (pxg_agg_stats)
  int32_t last_hc_reruns = 0; // partition passes the last finalize reran (pxg_agg_stats)
  int32_t EnsureHc(uint64_t need);
  // pxg_agg_finalize_result: result columns whose D2H copies the finalize issues as soon as
  // they are produced (keys on side stream 2, non-quantile values after the combine), so they
  // overlap the rest of the finalize.  cols has n_keys + n_udas entries; skip as in
  // pxg_agg_result_skip.
  struct EarlyResult {
    bool want = false, keys = false, vals = false;
    pxg_column_out* cols = nullptr;
    const uint8_t* skip = nullptr;
  } early;
  bool HcNext() const;     // would the next run after a reset be high-cardinality?
  int32_t FinalizeHc(struct HcExport* ex = nullptr);
  // Export of a high-cardinality run (pxg_hc.hip): partition groups' states after the table
  // groups' (states from g_table on), their key records as arena scratch named by eslots.
  int32_t ExportHcGroups(uint32_t g_table, DevBuf* states, DevBuf* eslots, uint32_t* n_hc, uint64_t* key_words);
  // Moves staged partition records into the table state (export / import need it): every
  // record's key goes to the arena and finds or inserts its group, its values become a staging
  // record.  No-op outside high-cardinality mode; afterwards the run continues on the table.
  int32_t SpillHc();

  AggResult res;
  DevBuf scratch;
  // Bumped by every consume / import / reset: export caches its partition per version.
  uint64_t state_version = 0;

  // Partial export workspace (pxg_partial.hip), valid for (n_parts, state_version).
  struct ExportCache {
    bool valid = false;
    int32_t n_parts = 0;
    uint64_t version = 0;
    DevBuf part_of, words, slist, grank, koff, rdigit, rlist, starts, hist, scan, scan2, desc, remap;
    bool v2 = false;  // the cache describes an exchange-v2 (partial states) export
    uint64_t G = 0;   // v2: groups of the export finalize
    std::vector<uint64_t> g_start, r_start, k_start;  // per part (+ total): groups, rows, key words
    // v2 group naming of the last export grouping: group g's key record at arena + (uint32_t)
    // e_slots[e_gslot[g]] (the table's slots / dense ids, or, for a high-cardinality run, eslots
    // with the partition groups' scratch records and an identity egslot); hc_key_words: the
    // scratch's words past arena_words.
    DevBuf eslots, egslot;
    const unsigned long long* e_slots = nullptr;
    const uint32_t* e_gslot = nullptr;
    uint64_t hc_key_words = 0;
    DevBuf dsend, dcnt;  // pxg_agg_export_partial_dev: the device-laid-out parts, their sizes and headers
  } xc;

  // Finalize workspace, kept across finalize calls (grow-only; no per-step allocation).
  struct FinalizeWs {
    DevBuf skey[2], sval[2][kMaxVals], rank;
    DevBuf hist, scan, scan2, cgroup, flags, gidx, meta, gstart, gslot, cbase, partial, lists;
    DevBuf keysA, keysB, bstarts, big, bchunks;
    // the designated big groups' own selection set (pxg_finalize.hip, started right after the
    // fused split's first pass): group / chunk lists, their list of ids and group starts,
    // counts (meta), chains, selection workspace
    struct EarlyBig {
      DevBuf big, chunks, ids, egs, meta, chain_starts, chain_nc;
      DevBuf spl, cnt, list, bstart, tag, cbase, plan, partial;
    } early;
    DevBuf fb_list, fb_meta;  // the fallback groups of both sets (full sort path)
    DevBuf chain_list, chain_nc, chain_starts;
    // big groups by selection (pxg_finalize.hip)
    DevBuf sel_spl, sel_cnt, sel_bstart, sel_tag, sel_cbase, sel_plan, sel_partial, sel_list, sel_bin;
    RadixPassWs rs;
    // high-cardinality finalize
    DevBuf hc_k[2], hc_v[2], hc_starts, hc_kscr, hc_meta;
    // staging split (pxg_finalize.hip): sampled slot counts, flag scan, bucket x tile counts,
    // bucket totals / bases
    DevBuf split_cnt, split_flags, split_hist, split_tot;
    DevBuf fs_keys;  // fused split: dense ids of the staged records (first pass)
    // export mode: per-group states, centroid lists of the big groups (kXCentCap per big group)
    // and their counts; owner side: merged digests' scratch, digest group list
    DevBuf xstates, xcent, xcnt, mrg, dlist;
  } ws;

  int32_t EnsureTable(uint32_t new_cap);
  int32_t EnsureStage(uint64_t need);
  int32_t Grow(uint32_t new_cap);
  int32_t PublishNew(Table* t, uint32_t* n_deferred);

  int32_t ConsumeRange(Table* t, int64_t begin, int64_t end);
  int32_t ConsumeList(Table* t, const uint32_t* list, uint32_t n);
  int32_t Finalize();
  int32_t PrepareExport(int32_t n_parts);
  int32_t ExportPartial(int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets, int64_t* part_bytes);
  int32_t ImportPartial(const void* src, int64_t nbytes);
  int32_t ImportPartials(const void* src, int32_t n, const int64_t* offs, const int64_t* sizes);
  // Exchange v2 (partial UDA states, pxg_partial.hip).
  int32_t ExportPartialV2(int32_t n_parts, void* dst, int64_t dst_capacity, int64_t* part_offsets, int64_t* part_bytes);
  int32_t ExportGroupV2(int32_t n_parts);
  int32_t CheckExportFinalize(const uint8_t* meta_copy);
  // pxg_agg_alltoall's export: parts laid out on the device (no host wait); per part its aligned
  // bytes to seg_dev[p] and its header to hdr_dev + 64 p.
  int32_t ExportPartialDev(int32_t n_parts, DevBuf* send, int64_t* seg_dev, uint8_t* hdr_dev);
  int32_t ImportPartialsV2(const uint8_t* base8, int32_t n, const int64_t* offs, const int64_t* sizes, const void* hdrs);
};

// Finalize stages (pxg_finalize.hip): the table path, then (high-cardinality mode) the
// partition records appended after its groups (pxg_hc.hip).
int32_t AggFinalizeImpl(Agg* agg);
int32_t AggFinalizeTable(Agg* agg);
// Merged digests of the groups listed in dlist (count on the device, at most cap_list) into
// every quantile UDA's output (pxg_finalize.hip; synchronises and checks its flags).
int32_t LaunchDigestMerge(Agg* a, const uint32_t* dlist, const uint32_t* dcount, uint32_t cap_list);
// Exchange v2 helpers (pxg_partial.hip): is the plan exchanging states; the accumulators of a
// merged aggregation following a table growth.
bool ExchangeV2(const Agg& a);
size_t XHeaderBytes();  // bytes of an exchange-v2 part header (the first bytes of every part)
int32_t MaccFollowGrow(Agg* a, const unsigned long long* old_slots, uint32_t old_cap, const uint32_t* remap, uint32_t new_cap);

// Groups the hint (or the last run) must reach before a qualifying plan stages partition
// records (PXG_HC_MIN_GROUPS overrides; tests use it at small sizes, 0 disables).
int64_t HcMinGroups();

}  // namespace pxg

struct pxg_agg {
  pxg::Agg impl;
};
