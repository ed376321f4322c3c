// cbf.hip -- the server's counting bloom filter (server/util/counting_bloom_filter.h,
// CountingBloomFilter<Key_t>) as batched gfx950 kernels.
//
// Counters: one u8 per index (m_bitarray, :60-65), padded with zeros to a
// multiple of kCbfChunk bytes so the pack pass reads whole chunks.  Index
// i of key x = (int)(murmur2(&x, 8, seed=i) % m) (ComputeHash :249-254),
// i < k; m < 2^31 keeps the int cast the identity.  Bitmap: MSB-first u64
// words, bit 63 - j%64 of word j/64 (ToOrdinaryBloomFilter :202-215), the
// format rdma_svr.cpp:157-251 ships and client/bloom_filter.c probes.
//
// Batch semantics equal the reference applied key by key in batch order:
//   Insert  (:109-118)  saturating += 1 per index.  Saturating increments
//           commute, so a per-byte CAS in any order gives the serial counters.
//   Delete  (:120-131)  if Query(x): -= 1 per index (uint8 wrap).  Order
//           matters only when a counter would reach zero under a later delete
//           of the same batch.  Fast path: query every key on the pre-batch
//           counters, then u32 atomicSub on the passing keys' bytes.  If no
//           subtraction ever sees its byte at 0, every counter c satisfied
//           c >= (decrements it received), so each key's serial query passed
//           too and the counters equal the serial result.  Otherwise (a flag
//           set on the device) the subtractions are added back (u32 add/sub
//           commute, borrows included) and one wave replays the batch in
//           order.  No host synchronisation either way.
#include "cceh_device.h"
#include "cceh_kernels.h"

#include <algorithm>

namespace pmdfc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t cbf_idx(uint64_t key, uint32_t salt, uint64_t m) {
  return (uint64_t)(murmur2_u64(key, salt) % (uint32_t)m);  // m < 2^31
}

__device__ __forceinline__ uint32_t* cbf_word(uint8_t* c, uint64_t idx) {
  return reinterpret_cast<uint32_t*>(c + (idx & ~3ull));
}

__device__ __forceinline__ uint32_t load_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Insert x n: lane per key, the k indices computed first so the k CAS chains
// are independent and overlap.  ops != nullptr: only keys whose op is
// PMDFC_OP_INSERT (1) count (KV::Insert's bf->Insert, server/KV.cpp:113-114).
__global__ __launch_bounds__(256) void k_cbf_insert(uint8_t* __restrict__ cnt, uint64_t m,
                                                    uint32_t k, const uint64_t* __restrict__ keys,
                                                    const uint8_t* __restrict__ ops, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if (ops && ops[i] != 1) return;
  const uint64_t key = keys[i];
  for (uint32_t j0 = 0; j0 < k; j0 += 4) {
    uint32_t* w[4];
    uint32_t sh[4], old[4];
    const uint32_t nj = min(4u, k - j0);
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      if (t < nj) {
        const uint64_t idx = cbf_idx(key, j0 + t, m);
        w[t] = cbf_word(cnt, idx);
        sh[t] = 8u * (uint32_t)(idx & 3u);
        old[t] = load_agent(w[t]);
      }
    }
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      if (t < nj) {
        uint32_t o = old[t];
        while (((o >> sh[t]) & 0xFFu) != 0xFFu) {
          const uint32_t prev = atomicCAS(w[t], o, o + (1u << sh[t]));
          if (prev == o) break;
          o = prev;
        }
      }
    }
  }
}

// Query x n (:133-143): lane per key, stops at the first zero counter.
__global__ __launch_bounds__(256) void k_cbf_query(const uint8_t* __restrict__ cnt, uint64_t m,
                                                   uint32_t k, const uint64_t* __restrict__ keys,
                                                   uint8_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  uint8_t r = 1;
  for (uint32_t j = 0; j < k; ++j) {
    if (cnt[cbf_idx(key, j, m)] == 0) {
      r = 0;
      break;
    }
  }
  out[i] = r;
}

// Delete, fast path.  undo = 0: subtract for every key whose pre-batch
// query (pass[]) held, flag a byte seen at 0; undo = 1 (acts only when
// flagged): add the same amounts back.
__global__ __launch_bounds__(256) void k_cbf_del_apply(uint8_t* __restrict__ cnt, uint64_t m,
                                                       uint32_t k, const uint64_t* __restrict__ keys,
                                                       const uint8_t* __restrict__ pass, uint64_t n,
                                                       uint32_t* __restrict__ flag, int undo) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if (undo && *flag == 0) return;
  if (!pass[i]) return;
  const uint64_t key = keys[i];
  bool hit0 = false;
  for (uint32_t j = 0; j < k; ++j) {
    const uint64_t idx = cbf_idx(key, j, m);
    const uint32_t sh = 8u * (uint32_t)(idx & 3u);
    if (undo) {
      atomicAdd(cbf_word(cnt, idx), 1u << sh);
    } else {
      const uint32_t o = atomicSub(cbf_word(cnt, idx), 1u << sh);
      hit0 |= ((o >> sh) & 0xFFu) == 0;
    }
  }
  if (hit0) *flag = 1u;
}

// Delete, serial replay (flagged batches only): one wave walks the batch in
// order; lane j < k owns index j of the current key.  Reads and CAS go to
// L2 (agent scope), so each key sees every earlier key's decrements.
__global__ __launch_bounds__(64) void k_cbf_del_serial(uint8_t* __restrict__ cnt, uint64_t m,
                                                       uint32_t k, const uint64_t* __restrict__ keys,
                                                       uint8_t* __restrict__ out, uint64_t n,
                                                       const uint32_t* __restrict__ flag) {
  if (*flag == 0) return;
  const uint32_t lane = threadIdx.x;
  const bool act = lane < k;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t key = keys[i];
    uint32_t* w = nullptr;
    uint32_t sh = 0, o = 0;
    bool zero = false;
    if (act) {
      const uint64_t idx = cbf_idx(key, lane, m);
      w = cbf_word(cnt, idx);
      sh = 8u * (uint32_t)(idx & 3u);
      o = load_agent(w);
      zero = ((o >> sh) & 0xFFu) == 0;
    }
    const bool ok = __ballot(zero) == 0;
    if (ok && act) {
      for (;;) {  // byte -= 1 (mod 256, no borrow), lanes sharing a word serialise
        const uint32_t nb = (((o >> sh) & 0xFFu) - 1u) & 0xFFu;
        const uint32_t nw = (o & ~(0xFFu << sh)) | (nb << sh);
        const uint32_t prev = atomicCAS(w, o, nw);
        if (prev == o) break;
        o = prev;
      }
    }
    if (lane == 0) out[i] = ok ? 1 : 0;
  }
}

// ToOrdinaryBloomFilter: each wave packs kCbfChunk (4 KiB) of counters per
// step.  Load r of lane l reads bytes [r*1024 + 16 l, +16) (one coalesced
// 1 KiB row per instruction); the 16 nonzero flags form 16 bits of word
// r*16 + l/4, a quad ORs its four parts, and lane l stores word
// (l&3)*16 + l/4 (one 512 B contiguous store per step).
__device__ __forceinline__ uint32_t nz_nibble(uint32_t x) {
  // byte b (little-endian) nonzero -> bit 3-b  (MSB-first within the nibble)
  const uint32_t t = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return ((t >> 4) & 8u) | ((t >> 13) & 4u) | ((t >> 22) & 2u) | (t >> 31);
}

__global__ __launch_bounds__(256) void k_cbf_pack(const uint8_t* __restrict__ cnt,
                                                  uint64_t* __restrict__ bm, uint64_t nwords,
                                                  uint64_t nchunks) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * 256u) >> 6;
  const uint32_t q = lane & 3u;
  for (uint64_t c = wave; c < nchunks; c += nwaves) {
    const u32x4* src = reinterpret_cast<const u32x4*>(cnt + c * kCbfChunk) + lane;
    u32x4 v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __builtin_nontemporal_load(src + r * 64);
    uint64_t mine = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t m16 = (nz_nibble(v[r].x) << 12) | (nz_nibble(v[r].y) << 8) |
                           (nz_nibble(v[r].z) << 4) | nz_nibble(v[r].w);
      uint64_t part = (uint64_t)m16 << (16u * (3u - q));
      part |= __shfl_xor(part, 1);
      part |= __shfl_xor(part, 2);
      if ((uint32_t)r == q) mine = part;
    }
    const uint64_t wi = c * (kCbfChunk / 64) + q * 16u + (lane >> 2);
    if (wi < nwords) bm[wi] = mine;
  }
}

#define GRID(n, per) dim3((unsigned)(((n) + (per)-1) / (per)))

void launch_cbf_insert(uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys,
                       const uint8_t* ops, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_cbf_insert, GRID(n, 256), dim3(256), 0, s, cnt, m, k, keys, ops, n);
}

void launch_cbf_query(const uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys,
                      uint8_t* out, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_cbf_query, GRID(n, 256), dim3(256), 0, s, cnt, m, k, keys, out, n);
}

void launch_cbf_delete(uint8_t* cnt, uint64_t m, uint32_t k, const uint64_t* keys, uint8_t* out,
                       uint64_t n, uint32_t* flag, hipStream_t s) {
  if (!n) return;
  (void)hipMemsetAsync(flag, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_cbf_query, GRID(n, 256), dim3(256), 0, s, cnt, m, k, keys, out, n);
  hipLaunchKernelGGL(k_cbf_del_apply, GRID(n, 256), dim3(256), 0, s, cnt, m, k, keys,
                     (const uint8_t*)out, n, flag, 0);
  hipLaunchKernelGGL(k_cbf_del_apply, GRID(n, 256), dim3(256), 0, s, cnt, m, k, keys,
                     (const uint8_t*)out, n, flag, 1);
  hipLaunchKernelGGL(k_cbf_del_serial, dim3(1), dim3(64), 0, s, cnt, m, k, keys, out, n,
                     (const uint32_t*)flag);
}

void launch_cbf_pack(const uint8_t* cnt, uint64_t m, uint64_t* bm, hipStream_t s) {
  const uint64_t nwords = (m + 63) / 64;
  const uint64_t nchunks = (m + kCbfChunk - 1) / kCbfChunk;
  const uint64_t blocks = std::min<uint64_t>((nchunks + 3) / 4, 4096);
  hipLaunchKernelGGL(k_cbf_pack, dim3((unsigned)blocks), dim3(256), 0, s, cnt, bm, nwords, nchunks);
}

}  // namespace pmdfc
