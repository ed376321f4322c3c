// cceh_kernels.h -- launcher declarations for cceh_kernels.hip / bloom.hip
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cceh_device.h"

namespace pmdfc {

void launch_get(bool count, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n, Geo g,
                const ulonglong2* pairs, uint32_t* partials, hipStream_t s);
// mixed batches: hash/reserved/shard check, mark the first insert of every
// touched segment, answer Gets that no earlier insert of the batch can affect
void launch_mixed_prep(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                       uint64_t n, Geo g, uint64_t* touched, uint64_t seq, hipStream_t s);
void launch_mixed_get(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                      uint64_t n, Geo g, const ulonglong2* pairs, const uint64_t* touched,
                      uint64_t seq, hipStream_t s);
void launch_init_segments(ulonglong2* pairs, uint32_t* occ, uint8_t* ldep, uint32_t* pool,
                          uint64_t* hdr, uint32_t nseg, uint32_t depth, uint32_t p1, hipStream_t s);
void launch_popcount(const uint32_t* occ, uint64_t nwords, unsigned long long* out, hipStream_t s);
void launch_hash(const uint64_t* keys, uint64_t* out, uint64_t n, hipStream_t s);
void launch_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, hipStream_t s);
void launch_owner(const uint64_t* keys, uint64_t n, uint32_t sbits, uint32_t* owner, uint32_t* idx,
                  hipStream_t s);
void launch_bounds(const uint32_t* sorted_owner, uint64_t n, uint32_t ngroups, uint64_t* starts,
                   hipStream_t s);

// bucket.hip (insert / mixed path)
constexpr uint32_t kPartTile = 4096;       // ops per partition block
constexpr uint32_t kMaxPartBlocks = 1024;  // => max_batch <= 4M
constexpr uint32_t kMaxP1 = 12;            // <= 4096 buckets
uint32_t part_blocks(uint64_t n);
struct PartLaunch {
  const uint64_t* keys;
  const uint64_t* vin;
  const uint8_t* ops;  // null: insert-only
  uint8_t* st;
  uint64_t n;
  uint32_t sbits, shard, p1, cap;
  uint64_t* rkey;
  uint64_t* rval;
  uint32_t* rop;
  uint32_t* cursor;
  uint2* runpos;
  DevCtl* ctl;
};
void launch_part(const PartLaunch& L, hipStream_t s);
struct BucketLaunch {
  uint64_t n;
  const uint64_t* rkey;
  const uint64_t* rval;
  const uint32_t* rop;
  const uint2* runpos;
  uint32_t chunk;
  uint32_t* cursor;
  uint64_t* hdr;
  uint32_t* pool;
  uint32_t pool_cap;
  uint32_t p1, sbits;
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  uint64_t* vout;
  uint8_t* st;
  uint32_t mixed;
  uint32_t max_segments;
  DevCtl* ctl;
};
void launch_bucket(const BucketLaunch& L, hipStream_t s);

// ubench.hip
void launch_gather64(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask,
                     uint64_t nops, uint64_t seed, uint64_t* out, hipStream_t s);

// bloom.hip
void launch_bloom_add(uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t n, hipStream_t s);
void launch_bloom_probe(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                        uint8_t* out, uint64_t n, hipStream_t s);
void launch_bloom_get(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t* vout, uint8_t* st, uint64_t n, Geo g, const ulonglong2* pairs,
                      hipStream_t s);

}  // namespace pmdfc
