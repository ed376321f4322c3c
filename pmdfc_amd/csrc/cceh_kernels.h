// cceh_kernels.h -- launcher declarations for cceh_kernels.hip / bloom.hip
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cceh_device.h"
#include "../../include/pmdfc_cceh.h"

namespace pmdfc {

// st == null: vout receives 16-B {value, status} records (routing responses)
void launch_get(bool count, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n, Geo g,
                const ulonglong2* pairs, uint32_t* partials, hipStream_t s);
// mixed batches, two exact ways (cceh_kernels.hip): the INSERT set --
// k_mixed_prep (every op's status, the batch's inserted keys in iset, ipos /
// icnt: per slot the key's insert position and a several-inserts flag) then
// k_mixed_get_iset (early answers; the Gets that need it probe the set) --
// or the JOIN -- k_mixed_get (statuses, early answers, the other Gets mark
// their keys' bits in jbits: status kStJoin), then k_mixed_join (the inserts
// whose bit is set put their keys into the set: per slot the count icnt and
// the first position ipos), then k_part resolves the kStJoin Gets.  early: 1 a
// single-copy hit, 2 linked to its insert (elink), 3 a non-wrapping
// single-copy hit.  A Get left pending sets ctl->pget = tag.  hint_ins:
// host-mapped, the batch's insert count (the host's choice of the next mode).
void launch_mixed_prep(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                       uint64_t n, Geo g, uint64_t* iset, uint64_t imask, uint32_t* ipos, uint32_t* icnt,
                       uint8_t* early, uint32_t* islot, DevCtl* ctl, uint32_t* loss0, uint32_t* icount,
                       hipStream_t s);
void launch_mixed_get_iset(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                           uint64_t n, Geo g, const ulonglong2* pairs, const uint64_t* iset, uint64_t imask,
                           const uint32_t* ipos, const uint32_t* icnt, uint8_t* early, uint32_t* elink, DevCtl* ctl,
                           uint32_t tag, uint32_t* icount, uint32_t ups, uint32_t* hint_ins, hipStream_t s);
void launch_mixed_get(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                      uint64_t n, Geo g, const ulonglong2* pairs, uint8_t* early, uint32_t* islot, uint32_t* jbits,
                      DevCtl* ctl, uint32_t* loss0, uint32_t tag, uint32_t* icount, uint32_t ups, hipStream_t s);
void launch_mixed_join(const uint8_t* ops, const uint64_t* keys, const uint8_t* st, uint64_t n,
                       uint64_t* iset, uint64_t imask, uint32_t* ipos, uint32_t* icnt, uint32_t* islot,
                       const uint32_t* jbits, DevCtl* ctl, uint32_t tag, const uint32_t* icount, uint32_t* hint_ins,
                       hipStream_t s);
// after the batch: linked Gets take their insert's outcome; early hits whose
// key a split of the batch dropped are placed before / after that split's
// insert through the drop log (PMDFC_ST_SPLIT_LOST only if the log overflowed)
void launch_mixed_verify(const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint8_t* st, uint64_t* vout,
                         uint64_t n, Geo g,
                         const ulonglong2* pairs, const uint8_t* early, const uint32_t* elink, DevCtl* ctl,
                         const uint32_t* loss0, const ulonglong2* drops, uint64_t* iset, uint32_t* icnt,
                         uint32_t* ipos, const uint32_t* islot, uint64_t imask, uint32_t* jbits /* null: insert set */,
                         hipStream_t s);
// upsert batches: pre-batch slot of each Insert's key (0xFFFF absent); ops may
// be null (insert-only), kvs = u64 words from one key to the next
void launch_upsert_probe(const uint64_t* keys, uint32_t kvs, const uint8_t* ops, uint64_t n, Geo g,
                         const ulonglong2* pairs, uint16_t* upos, hipStream_t s);
// the smallest live local depth -> *out (set to ~0 before)
void launch_min_ldep(const uint8_t* ldep, const DevCtl* ctl, uint32_t max_segs, uint32_t* out, hipStream_t s);
// directory buckets p1 -> p1n bits (every segment's local depth >= sbits + p1n)
void launch_rebucket(const uint64_t* old_hdr, uint64_t* hdr, uint32_t p1, uint32_t p1n, hipStream_t s);
// Fixed sub-directory slots: once the table is at its final bucket resolution
// (p1 == p1max: the bucket numbering never changes again), a sub-directory of
// at most 2^kFixedBits entries lives at pool offset w * kFixedSlot, the pool
// region [0, 2^p1max * kFixedSlot) being reserved for them, and grows there in
// place.  The first apply pass then loads it speculatively with the bucket's
// header and records (one dependent round trip less) and keeps it if the
// header points there.  Everything else is allocated past that region.
// (128 entries: a 2^28-key table at 2^13 buckets has sub-directories of
// 64-128 entries; 2 MiB of pool per 2^14 buckets.)
constexpr uint32_t kFixedBits = 7;
constexpr uint32_t kFixedSlot = 1u << kFixedBits;
// fixed: the initial sub-directories go to their fixed slots (p1 == p1max and
// db0 <= kFixedBits); else to the pool at `region`
// the control block of a fresh table (and the host-mapped hint), in stream order
// word arrays a reset zeroes in k_init_segments' launch (p[k]: n[k] u32 words)
constexpr int kInitZero = 6;
struct InitZero {
  uint32_t* p[kInitZero];
  uint64_t n[kInitZero];
};
void launch_init_segments(ulonglong2* pairs, uint32_t* occ, uint8_t* ldep, uint32_t* pool,
                          uint64_t* hdr, uint32_t nseg, uint32_t depth, uint32_t p1, uint32_t fixed,
                          uint32_t region, const InitZero& z, DevCtl* ctl, uint32_t pool_cur, uint32_t* hint,
                          hipStream_t s);
// flatten the bucketed directory for pure-Get batches: *bits = p1 + max db
// (the physical depth), flat[x] = the sub-directory entry of index x
void launch_flatten(const uint64_t* hdr, const uint32_t* pool, uint32_t p1, uint32_t* flat,
                    uint32_t* bits, uint32_t max_bits, hipStream_t s);
void launch_popcount(const uint32_t* occ, uint64_t nwords, unsigned long long* out, hipStream_t s);
// CCEH::FindAnyway x n: first copy of each key in slot order (wave per key)
void launch_find_anyway(const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n, Geo g,
                        const ulonglong2* pairs, hipStream_t s);
void launch_hash(const uint64_t* keys, uint64_t* out, uint64_t n, hipStream_t s);
void launch_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, hipStream_t s);
void launch_owner(const uint64_t* keys, uint64_t n, uint32_t sbits, uint32_t* owner, uint32_t* idx,
                  hipStream_t s);
void launch_bounds(const uint32_t* sorted_owner, uint64_t n, uint32_t ngroups, uint64_t* starts,
                   hipStream_t s);

// bucket.hip (insert / mixed path)
constexpr uint32_t kPartTile = 8192;       // ops per partition block (A/B: 4096 32.4 us per 1M, 8192 30.9, 16384 57)
constexpr uint32_t kMaxPartBlocks = 512;   // => max_batch <= 4M
constexpr uint32_t kMaxP1 = 14;            // <= 16384 directory buckets
constexpr uint32_t kServeWavesMax = 64;     // serving waves (PMDFC_SERVE_WAVES_MAX)
constexpr uint32_t kCpSbb = 3;             // coarse partition: 8 directory buckets per partition bucket
constexpr uint32_t kMaxPartBits = 13;      // <= 8192 partition buckets
// A partition bucket's record region is cut into kPartSubs sub-regions, one
// per XCD-sharing class of k_part blocks (blocks b and b + 8 share an XCD,
// MI355X_MICROARCH.md "Workgroup dispatch"): block b writes sub-region b % 8
// only, so every line of a sub-region is dirtied in ONE XCD's L2 and leaves
// it whole, and each region cursor is bumped by 1/8 of the blocks.
constexpr uint32_t kPartSubs = 8;
uint32_t part_blocks(uint64_t n);
struct PartLaunch {
  const uint64_t* keys;
  const uint64_t* vin;
  const uint8_t* ops;  // null: insert-only
  uint8_t* st;
  uint64_t n;
  uint32_t kvs;        // key/value stride in u64 words (0/1: arrays; 2: {key, value} records)
  uint32_t sbits, shard;
  uint32_t p1, sbb;    // directory bucket bits, of which sbb sub-bucket bits
  uint32_t cap;        // record slots per partition bucket
  ulonglong2* rkv;
  uint32_t* rop;
  uint16_t* robk;
  uint32_t* cursor;    // this batch's parity
  uint32_t* ovf;
  uint32_t* povf;      // [tile][partition bucket] overflow slots (this batch's parity)
  uint64_t* stamps;    // debug phase stamps or null
  // a medium mixed batch (one partition block, k_medium after): statuses
  // initialized here (k_mixed_prep's rule), Get values zeroed, and the
  // partition buckets that received ops listed ([0] count, then the buckets)
  uint32_t init;
  uint64_t* vout;
  uint32_t* touched;
  // a general mixed batch: its joining Gets (kStJoin) are resolved here from
  // the join's per-slot counts (k_mixed_get, k_mixed_join)
  const uint64_t* iset;
  uint64_t imask;
  const uint32_t* icnt;
  const uint32_t* ipos;
  uint8_t* early;
  uint32_t* elink;
  DevCtl* ctl;
  uint32_t tag;
};
void launch_part(const PartLaunch& L, hipStream_t s);
struct BucketLaunch {
  uint64_t n;
  const ulonglong2* rkv;
  const uint32_t* rop;
  const uint16_t* robk;
  uint32_t chunk;
  uint32_t cap;       // records per partition bucket region (kPartSubs sub-regions of cap / kPartSubs)
  const uint32_t* cursor;  // [kPartSubs][partition buckets] cursors, then the overflow cursor
  const uint32_t* ovf;
  uint32_t* cursor_next;
  uint32_t* ovf_next;
  uint32_t clear_next;  // first apply pass zeroes the other parity's cursors (one batch per call)
  uint64_t* hdr;
  uint32_t* pool;
  uint32_t pool_cap;
  uint32_t p1, sbb, sbits, shard;
  uint32_t pfix;      // p1 == p1max: small sub-directories live (and grow) in their fixed slots
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  uint64_t* vout;
  uint8_t* st;
  uint32_t mixed;
  uint32_t upsert;    // last-writer-wins Insert (PMDFC_CFG_UPSERT)
  const uint16_t* upos;  // upsert: pre-batch slot of each op's key (k_upsert_probe), first pass only
  uint32_t max_segments;
  DevCtl* ctl;
  uint64_t* wstat;    // per directory bucket stat slots (kWStat each)
  ulonglong2* wl_kv;  // parked ops: kChunkWave per directory bucket
  uint32_t* wl_op;
  uint32_t* wl_n;
  uint64_t* stamps;  // debug phase stamps or null
  // pipelined split rounds (an apply pass requests and grants -> k_split)
  uint2* req;        // kSplitCap split requests per directory bucket
  uint32_t* reqop;   // ... the batch position of each request's insert
  ulonglong2* drops; // mixed batches with early answers: the drop log (cceh_device.h kDropLog), else null
  uint32_t* need;    // per bucket: sub-directory bits those requests need (0: none)
  uint32_t* gbase;   // per bucket: first child segment id granted
  uint32_t* ngrant;  // per bucket: requests granted, committed by the owner's next pass
  uint32_t* newoff;  // per bucket: pool offset of the grown sub-directory
  uint64_t* gsh;     // [2][kGShards] grant shard words by batch parity (kGStride apart)
  uint4* gsplit;     // [2][kGShards][gcap] the requested splits by segment offset in their shard:
                     // {request word, w | i << 14 | entry << 20, pool offset, nr | need << 8}
  uint32_t gcap;     // splits per shard (kSplitCap x the shard's buckets)
  uint32_t* act;     // [2^p1] buckets with requests (k_split -> k_apply_parked)
  uint32_t* fbl;     // [2^p1max] per bucket: declined by k_apply_fast (bit 0), decline count (bits 1+)
  uint64_t* split_stamps;  // debug: 8 stamps for each of the first kSplitStamps splits, or null
  // worklists: the passes after k_apply visit only the buckets that have work
  uint32_t* fin;     // [2][2^p1] by batch parity: buckets for the final pass
  uint32_t par;      // this batch's parity
  uint32_t gate_tag; // mixed batches: != 0 lets the insert-only apply passes run unless ctl->pget == gate_tag
  // gated mixed batches: the host expects the mixed passes to stay gated off
  // (no recent batch ran them, mseen) and launches them on small looping
  // grids, so their exit costs less; mseen: the host-mapped word the first
  // mixed pass stamps with gate_tag when it runs
  uint32_t mixed_small;
  uint32_t* mseen;
  uint32_t wide;     // the lean first pass in its wide variant (k_apply_wide: sub-directories up to 128 entries)
  uint32_t fb;       // launch k_apply_fb after it (else k_apply_parked takes the declined buckets)
  uint32_t cp;       // coarse partition (sbb == 3): the lean first pass is k_apply_fast_cp
  uint32_t* hint;    // device-mapped pinned word: k_apply_parked leaves the segment count there (host hint)
  uint32_t ramp = 0;  // the table still ramps (p1 < p1max) or is small for the batch: the larger grids
};
constexpr uint32_t kSplitStamps = 8192;
// Split requests are granted through kGShards pairs of counters, one per XCD
// (bucket w -> shard w % 8, the XCD its first-pass wave runs on), each word
// on a 128-B line of its own: {child segments [0,32) | requesting buckets
// [32,64)} and the sub-directory pool entries requested in this batch.  A
// contended single word serializes at ~88 atomics/us, far below the rate of
// a split-heavy batch's ~8k requests.
constexpr uint32_t kGShards = 8;
constexpr uint32_t kGStride = 32;  // u64 words per shard: the segment word at 0, the pool word at 16
constexpr uint32_t kChunkWave = 256;  // ops per k_apply / k_bucket wave chunk (mean load: 128)
constexpr uint32_t kSplitCap = 64;    // split requests per directory bucket and round
// per-bucket cumulative counters: lines, waited, splits, split loss, runs,
// rounds, {max rounds | max local depth << 16 | growths << 32}, spare
constexpr int kWStat = 8;
// k_apply: mode 0 = first pass over the batch's records, 1 = pass over the
// parked ops (after a split round); final: k_bucket (inline splits, the rest)
void launch_apply(const BucketLaunch& L, uint32_t mode, hipStream_t s);
// the lean first pass is on (PMDFC_FAST_APPLY=0 turns it off: A/B)
bool fast_first_pass();
// k_apply_fb after the lean first pass (insert-only batches; nothing otherwise)
void launch_apply_fallback(const BucketLaunch& L, hipStream_t s);
void launch_final(const BucketLaunch& L, hipStream_t s);
// a batch of at most kPartTile ops after its one-block partition (k_part with
// a touched list): every listed partition bucket's directory buckets through
// the final pass, records walked in batch order (k_medium)
void launch_medium(const BucketLaunch& L, const uint32_t* touched, hipStream_t s);
// the persistent serving kernel of the per-op front-end (k_serve, one wave)
struct ServeLaunch {
  const pmdfc_serve_req* req;  // device mappings of the host rings
  pmdfc_serve_resp* resp;
  pmdfc_serve_ctl* ctl;
  uint64_t ring_size, head0;
  uint8_t* cbf;
  uint64_t cbf_m;
  uint32_t cbf_k;
  uint32_t nwaves;  // 0/1: one wave from head0; else wave w serves ring w from ctl[w].head
};
void launch_serve(const BucketLaunch& L, const ServeLaunch& V, hipStream_t s);
// a whole batch of n <= kChunkWave ops in one launch (k_mixed_small); ops ==
// null: insert-only.  L.st / L.vout are the outputs; inputs may be host-mapped
void launch_mixed_small(const BucketLaunch& L, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                        hipStream_t s);
// one split round: split every segment the apply pass granted (it hands out
// child ids / sub-directory space itself), one wave each (k_split)
// insert-only batches: the split round and the last parked pass in one launch
void launch_split_round(const BucketLaunch& L, hipStream_t s);

// ubench.hip
void launch_gather64(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask,
                     uint64_t nops, uint64_t seed, uint64_t* out, hipStream_t s);
int launch_gather(const void* buf, uint64_t nbytes, uint32_t line, uint32_t depth, const uint32_t* table,
                  uint32_t tmask, uint64_t nops, uint64_t seed, uint64_t* out, uint64_t omask, hipStream_t s);
int launch_scatter16(void* buf, uint64_t nbytes, uint32_t depth, uint64_t nops, uint64_t seed, hipStream_t s);

// bloom.hip
void launch_bloom_add(uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t n, hipStream_t s);
void launch_bloom_probe(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                        uint8_t* out, uint64_t n, hipStream_t s);
void launch_bloom_get(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t* vout, uint8_t* st, uint64_t n, Geo g, const ulonglong2* pairs,
                      hipStream_t s);

// cbf.hip (server counting bloom filter, counting_bloom_filter.h)
constexpr uint64_t kCbfChunk = 4096;  // counter bytes per pack step (counters padded to it)
void launch_cbf_insert(uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys,
                       const uint8_t* ops, uint64_t n, hipStream_t s);
void launch_cbf_query(const uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys,
                      uint8_t* out, uint64_t n, hipStream_t s);
void launch_cbf_delete(uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys, uint8_t* out,
                       uint64_t n, uint32_t* flag, hipStream_t s);
void launch_cbf_pack(const uint8_t* cnt, uint64_t m, uint64_t* bm, hipStream_t s);

// trace.hip (replay_KV trace ingestion)
struct TraceLine {
  uint64_t key;  // (inode << 32) + offset
  uint32_t op;   // PMDFC_OP_INSERT (W) / PMDFC_OP_GET (R, or no ops)
  uint32_t pad;
};
uint64_t trace_nl_tiles(uint64_t nbytes);
size_t trace_scan_temp_bytes(uint64_t nlines);
hipError_t launch_trace_newlines(const char* text, uint64_t nbytes, uint64_t* nl, uint64_t* d_nnl,
                                 uint64_t* tile_cnt, uint64_t* tile_off, void* temp,
                                 size_t temp_bytes, hipStream_t s);
hipError_t launch_trace_lines(const char* text, uint64_t nbytes, const uint64_t* nl, uint64_t nnl,
                              uint64_t nlines, TraceLine* lines, uint64_t* pages, uint64_t* cum,
                              unsigned long long* first_bad, uint64_t num_data, uint64_t* info,
                              void* temp, size_t temp_bytes, hipStream_t s);
void launch_trace_expand(const TraceLine* lines, const uint64_t* cum, const uint64_t* pages,
                         uint64_t nlines, uint64_t nout, uint8_t* ops, uint64_t* keys,
                         hipStream_t s);

// extent.hip (Insert_extent / Get_extent, both reference variants)
hipError_t launch_extent_count(bool src, const uint64_t* keys, const uint64_t* cl, const uint64_t* lens,
                               uint64_t n, uint64_t* cnt, uint64_t* cum, hipStream_t s);
void launch_extent_expand(bool src, const uint64_t* keys, const uint64_t* cl, const uint64_t* lens,
                          const uint64_t* vals, uint64_t n, const uint64_t* cum, uint64_t* out_k,
                          uint64_t* out_v, hipStream_t s);
uint32_t extent_targets_per_key(bool src);
void launch_extent_targets(const uint64_t* keys, const uint64_t* cl, uint64_t n, uint32_t per,
                           uint64_t* out, hipStream_t s);
void launch_extent_pick(const uint64_t* v, const uint8_t* st, uint64_t n, uint32_t per, uint64_t* vout,
                        uint8_t* sout, hipStream_t s);

// route.hip (multi-GPU: fixed-capacity owner blocks for equal-split
// all-to-alls, with a per-owner carry so no op is ever dropped)
constexpr uint32_t kRouteTile = 1024;     // ops per routing block
constexpr uint32_t kRouteMaxOwners = 16;  // shard_bits <= 4
constexpr uint32_t kRouteNone = 0xFFFFFFFFu;  // rowpos of a padding row
constexpr uint32_t kCarryWords = 3;       // carried records: key, value, op (width <= 3 used)
struct RouteArgs {
  const uint64_t* keys;
  const uint64_t* vals;  // width >= 2
  const uint8_t* ops;    // width 3
  const uint8_t* keep;   // nullable: ops with keep[i] == 0 stay home (ST_FILTERED)
  uint64_t n;
  uint32_t sbits;
  uint32_t width;        // u64 words per record: key[, value[, op]]
  uint64_t cap;          // record slots per owner block
  uint64_t cc;           // carry slots per owner
  uint32_t base;         // call-global output index of op 0
  uint64_t* send;        // [2^sbits][cap][width]
  uint32_t* rowpos;      // [2^sbits * cap] call-global output index of the row, or kRouteNone
  uint64_t* vals_out;    // nullable, call-global: 0 for ops that are not sent
  uint8_t* st_out;       // call-global: ST_FILTERED / ST_ROUTE_OVERFLOW for ops that are not sent
  uint32_t* tile_cnt;    // [route_tiles(n)][2^sbits]
  const uint32_t* cin;   // [2^sbits] ops carried in (the previous pack's cout)
  uint32_t* cout;        // [2^sbits] ops carried out
  const uint64_t* crec_in;   // [2^sbits][cc][kCarryWords]
  uint64_t* crec_out;
  const uint32_t* cpos_in;   // [2^sbits][cc] call-global output index
  uint32_t* cpos_out;
  uint32_t* ovf;         // ops dropped because the carry was full (sticky count)
  // the local block: owner self_g's rows go to self_dst ([cap][width], the
  // receive buffer's slot for this rank) instead of send (null: send)
  uint32_t self_g;
  uint64_t* self_dst;
};
uint32_t route_tiles(uint64_t n);
void launch_route_pack(const RouteArgs& a, hipStream_t s);
void launch_route_split(const uint64_t* recv, uint64_t rows, uint32_t W, uint64_t* keys, uint64_t* vals,
                        uint8_t* ops, hipStream_t s);
void launch_route_resp(const uint64_t* vals, const uint8_t* st, uint64_t rows, void* resp, hipStream_t s);
// rows [self_lo, self_hi) are read from back_self (the local block's
// responses where the engine wrote them), the others from back
void launch_route_unpack(const void* back, uint32_t W, const uint32_t* rowpos, uint64_t rows, uint64_t* vals_out,
                         uint8_t* st_out, hipStream_t s, const void* back_self = nullptr, uint64_t self_lo = 0,
                         uint64_t self_hi = 0);
void launch_route_carried(const uint32_t* cnt, uint32_t G, uint64_t* out, hipStream_t s);
// Get dedupe within tiles of 4096 Gets (LDS table)
void launch_route_dedupe(const uint64_t* keys, const uint8_t* keep_in, uint64_t n, uint32_t base, uint8_t* keep_out,
                         uint32_t* lead_out, hipStream_t s);
void launch_route_fill(const uint32_t* lead, uint64_t n, uint64_t* vals, uint8_t* st, hipStream_t s);

}  // namespace pmdfc
