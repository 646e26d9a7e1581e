// Hash group-by aggregation (AggNode, src/carnot/exec/agg_node.cc:88-542) on MI355X.
//
// Design: the fused consume kernel evaluates the filter, the group-key hash and
// the UDA argument expressions per row and appends one staging record (slot, values) per
// selected row; group identity is a slot of a global open-addressing table whose 64-bit slot
// words are only ever written by CAS and read by agent-scope atomic loads (no cross-workgroup
// plain-data hand-off inside a launch).  Finalize sorts the staging by slot (stable LSD radix
// sort), reduces each run (count/sum/mean/min/max) and builds each group's t-digest from its
// sorted values (QuantilesUDA semantics).
#pragma once

#include "pxg_internal.h"

namespace pxg {

// Slot word layout: [63:33] tag (31 bits, never 0) | [32] kind | [31:0] ref.
//   kind 0: ref = (chunk << 24) | local row of the table consumed by the current launch
//   kind 1: ref = 8-byte word offset of the key record in the agg's key arena
constexpr uint64_t kKindArena = 1ULL << 32;
constexpr uint32_t kDeferredSlot = 0xFFFFFFFFu;
// Bytes kept allocated past the last key record: the consume fast path loads a whole key
// record speculatively (at most kMaxKeys * 7 words) before it knows the record's length.
constexpr uint64_t kArenaSlack = 512;

__device__ __forceinline__ uint32_t SlotTag(uint64_t h) { return static_cast<uint32_t>((h >> 33) | 1u) & 0x7FFFFFFFu; }
__device__ __forceinline__ uint64_t MakeSlotWord(uint32_t tag, uint64_t kind, uint32_t ref) {
  return (static_cast<uint64_t>(tag) << 33) | kind | ref;
}

enum ValKind : int32_t { kValProgram = 0, kValMinOf2 = 1 };

struct AggPlanDev {
  int32_t n_keys;
  int32_t n_udas;
  int32_t n_vals;
  int32_t has_filter;
  int32_t key_types[kMaxKeys];
  int32_t uda_kind[kMaxUdas];
  int32_t uda_val[kMaxUdas];   // staged stream index (-1: none)
  int32_t uda_arg_type[kMaxUdas];
  int64_t uda_init[kMaxUdas];   // init arg (MINSUM) or 0
  int32_t uda_val2[kMaxUdas];  // second staged stream (MEAN_MERGE: the state sizes) or -1
  int32_t state_off[kMaxUdas]; // emit_states: byte offset of the UDA's Serialize() bytes
  int32_t state_rec;           // emit_states: bytes per group record (0: no states)
  int32_t emit_states;
  int32_t val_kind[kMaxVals];
  int32_t val_type[kMaxVals];   // result type of the stream (INT64/TIME64NS/FLOAT64/BOOLEAN)
  int32_t col_types[kMaxCols];
  DevProgram filter;
  DevProgram keys[kMaxKeys];
  DevProgram vals[kMaxVals];
  DevProgram vals2[kMaxVals];
};

// Probe records (consume fast path, all-STRING keys, <= 2 keys): per table slot kRecWords
// words = [the published slot word, the key lengths (16 bits per key), key 0's kRecKeyWords
// words, key 1's ...], tail-masked and zero-padded, 128-byte aligned.  Written by publication
// (and rebuilt after a rehash); a probe that meets a published (arena) slot word compares its
// keys against the record at the same position with 16-byte loads of one line instead of the
// arena / representative row.  Word 0 equal to the slot word the probe saw
// is what makes a record valid: records are cleared at reset and rebuilt after growth.
constexpr int kRecWords = 16;
constexpr int kRecKeyWords = 6;  // = kFastStrWords: STRING keys of <= 48 bytes
constexpr int kRecMaxKeys = 2;

struct AggTableDev {
  unsigned long long* slots;
  uint64_t* prec;  // probe records (null: off); row-record consumes also write them
  uint32_t mask;
  uint32_t limit;                 // inserts beyond this are deferred (table kept <= 50% full)
  unsigned int* counters;         // [0] groups in the table (flushed per tile), [2] deferred rows
  uint32_t* deferred;      // rowrefs of deferred rows
  uint32_t* deferred_pos;  // their staging records (the retry fills in the slot)
  const uint64_t* arena;
};

// High-cardinality (partitioned) staging, pxg_hc.hip: one record per selected row whose keys
// fit, stored as `stride` word streams (stream j of record i at rec[j * cap + i], so the consume
// kernel's stores and the partition sort's loads are coalesced): word 0 holds the STRING key
// lengths (16 bits per key; ~0 marks a hole left by a row that took the table path), then every
// key's words (tail-masked), then the value streams.  key[i] = the top half of the key hash
// (partition bits on top).
constexpr int kHcStrWords = 3;  // STRING keys of <= 24 bytes ride in the record
constexpr int kHcMaxVals = 4;
constexpr int kHcMaxStride = 16;  // record streams the partition sort moves (kMaxVals)
constexpr uint64_t kHcHole = ~0ULL;
constexpr int kHcTableEntries = 1024;  // LDS table entries per partition (pxg_hc.hip kHcTable)
// Dynamic LDS of one hc_agg workgroup: per table entry an 8-byte {tag, record}, 8 bytes per
// accumulator and per MEAN high word (the exact 128-bit sum), and a 4-byte count.
inline size_t HcAggLdsBytes(int n_acc, int n_wide) { return static_cast<size_t>(kHcTableEntries) * (8 + 8 * (n_acc + n_wide) + 4); }
// What hc_agg may declare: gfx950 gives one workgroup up to 160 KiB of LDS; a margin is left for
// the kernel's static LDS.
inline size_t HcMaxDynLds() { return static_cast<size_t>(144) << 10; }

struct HcStageDev {
  uint64_t* rec;
  uint32_t* key;
  unsigned long long* cursor;
  unsigned int* maxlen;  // [kMaxKeys]: the longest STRING key staged (finalize sorts only its words)
  uint64_t cap;  // words per stream
  int32_t stride, kwords;
  int32_t kw[kMaxKeys], koff[kMaxKeys];
};

struct StageDev {
  uint32_t* slot;
  uint64_t* vals[kMaxVals];
  unsigned long long* cursor;
  HcStageDev hc;
};

}  // namespace pxg
