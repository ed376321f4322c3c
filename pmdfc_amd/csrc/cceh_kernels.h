// cceh_kernels.h -- launcher declarations for cceh_kernels.hip / bloom.hip
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cceh_device.h"

namespace pmdfc {

void launch_get(bool count, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n, Geo g,
                const ulonglong2* pairs, uint32_t* partials, hipStream_t s);
void launch_prep(const uint64_t* keys, uint64_t* hbuf, uint8_t* st, uint64_t* vout, uint64_t n,
                 uint32_t sbits, uint32_t shard, hipStream_t s);
void launch_mark(const uint8_t* ops, const uint64_t* hbuf, const uint8_t* st, uint64_t n, Geo g,
                 uint8_t* touched, hipStream_t s);
void launch_mixed_get(const uint8_t* ops, const uint64_t* keys, const uint64_t* hbuf, uint8_t* st,
                      uint64_t* vout, uint64_t n, Geo g, const ulonglong2* pairs,
                      const uint8_t* touched, uint8_t* pend_flag, hipStream_t s);
void launch_route(const uint32_t* pend, uint64_t npend, const uint64_t* hbuf, const uint8_t* st,
                  Geo g, uint32_t sent, uint32_t* skey, uint32_t* sval, hipStream_t s);
void launch_process(const uint32_t* skey, const uint32_t* sval, uint64_t npend, uint32_t sent,
                    const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint64_t* vout,
                    uint8_t* st, const uint64_t* hbuf, ulonglong2* pairs, uint32_t* occ,
                    const uint8_t* ldep, uint8_t* deferred, uint32_t* split_list, DevCtl* ctl,
                    uint32_t gdepth, uint32_t max_segments, hipStream_t s);
void launch_split(uint32_t nsplit, const uint32_t* split_list, ulonglong2* pairs, uint32_t* occ,
                  uint8_t* ldep, uint32_t* dir, uint32_t gdepth, uint32_t sbits, DevCtl* ctl,
                  hipStream_t s);
void launch_double(const uint32_t* od, uint32_t* nd, uint64_t n_new, hipStream_t s);
void launch_init_segments(ulonglong2* pairs, uint32_t* occ, uint8_t* ldep, uint32_t* dir,
                          uint32_t nseg, uint32_t depth, hipStream_t s);
void launch_popcount(const uint32_t* occ, uint64_t nwords, unsigned long long* out, hipStream_t s);
void launch_hash(const uint64_t* keys, uint64_t* out, uint64_t n, hipStream_t s);
void launch_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, hipStream_t s);
void launch_owner(const uint64_t* keys, uint64_t n, uint32_t sbits, uint32_t* owner, uint32_t* idx,
                  hipStream_t s);
void launch_bounds(const uint32_t* sorted_owner, uint64_t n, uint32_t ngroups, uint64_t* starts,
                   hipStream_t s);

// bucket.hip (fast insert/mixed path)
constexpr uint32_t kBucketPasses = 3;
uint32_t part_blocks(uint64_t n);
void launch_part_hist(const uint32_t* pend, const uint32_t* npend_dev, uint64_t npend_host,
                      uint64_t nmax, const uint8_t* st, const uint64_t* hbuf, uint32_t sbits,
                      uint32_t p1, uint32_t* hist, hipStream_t s);
void launch_part_scatter(const uint32_t* pend, const uint32_t* npend_dev, uint64_t npend_host,
                         uint64_t nmax, const uint8_t* st, const uint64_t* hbuf, uint32_t sbits,
                         uint32_t p1, uint32_t bbits, const uint32_t* hist, const uint32_t* inc,
                         uint64_t* rec, hipStream_t s);
struct BucketLaunch {
  const uint64_t* rec;
  const uint32_t* inc;  // inclusive scan of the partition histogram
  uint64_t nmax;
  uint32_t p1, bbits, gdepth, sbits, pass, last;
  const uint8_t* ops;
  const uint64_t* keys;
  const uint64_t* vin;
  uint64_t* vout;
  uint8_t* st;
  ulonglong2* pairs;
  uint32_t* occ;
  const uint32_t* dir;
  uint8_t* pstate;
  uint8_t* bwork;
  uint8_t* hostdef;
  uint32_t* split_list;
  DevCtl* ctl;
  uint32_t max_segments;
};
void launch_bucket(const BucketLaunch& L, hipStream_t s);
void launch_split_q(const uint32_t* split_list, const uint32_t* count, ulonglong2* pairs,
                    uint32_t* occ, uint8_t* ldep, uint32_t* dir, uint32_t gdepth, uint32_t sbits,
                    DevCtl* ctl, uint32_t grid, hipStream_t s);

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
