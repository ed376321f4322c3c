// cceh_kernels.hip -- hand-written gfx950 kernels of the batched CCEH engine:
// the Get path (one quad per key), the mixed-batch pre-pass, table init and
// small utilities.  The Insert path (partition + per-bucket apply/split) is in
// bucket.hip.
//
// Batch semantics: ops are applied as if run serially in batch
// order on CCEH_hybrid.  A segment's contents depend only on the subsequence
// of ops whose hash falls in its key range, so each segment's ops are applied
// in batch order by one lane, segments in parallel.
#include "cceh_device.h"
#include "cceh_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace pmdfc {

// ---------------------------------------------------------------- get path
// Pure-Get batch: 4 lanes per key, 64 keys per 256-thread block.
template <bool COUNT>
__global__ __launch_bounds__(256) void k_get(const uint64_t* __restrict__ keys,
                                             uint64_t* __restrict__ vout,
                                             uint8_t* __restrict__ st, uint64_t n, Geo g,
                                             const ulonglong2* __restrict__ pairs,
                                             uint32_t* __restrict__ line_partials) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  uint32_t lines = 0;
  if (op < n) {
    const uint64_t key = keys[op];
    const uint64_t h = hash64(key);
    uint64_t val = 0;
    uint8_t s;
    if (reserved_key(key)) {
      s = 3;  // PMDFC_ST_RESERVED_KEY
    } else if (wrong_shard(h, g.sbits, g.shard)) {
      s = 8;  // PMDFC_ST_WRONG_SHARD
    } else {
      const uint32_t seg = de_seg(dir_entry(g, h));
      s = quad_probe(pairs + (size_t)seg * kSlots, key, h, q, &val, &lines);
    }
    if (q == 0) {
      if (st) {
        vout[op] = val;
        st[op] = s;
      } else {  // routing response record
        reinterpret_cast<ulonglong2*>(vout)[op] = make_ulonglong2(val, (unsigned long long)s);
      }
    }
  }
  if (COUNT) {
    __shared__ uint32_t red[4];
    uint32_t v = (q == 0) ? lines : 0;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) line_partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

// Pure-Get batch, U independent keys per quad (ops q, q+Q, q+2Q, ... with Q =
// quads in the grid): the U key loads, directory loads and first window-line
// loads are issued back to back, so each wave keeps U x 16 random lines in
// flight instead of 16.  Most Gets finish on the first line (L ~ 1.02); the
// rest continue one key at a time.
template <int U, bool COUNT>
__global__ __launch_bounds__(256) void k_get_u(const uint64_t* __restrict__ keys,
                                               uint64_t* __restrict__ vout,
                                               uint8_t* __restrict__ st, uint64_t n, Geo g,
                                               const ulonglong2* __restrict__ pairs,
                                               uint32_t* __restrict__ line_partials, uint32_t p2on,
                                               uint32_t rounds) {
  const uint64_t nq = (uint64_t)gridDim.x * 64u;
  const uint64_t q0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t qbase = (threadIdx.x & 63u) & ~3u;
  uint32_t lines = 0;
  // (a capped grid: every quad takes `rounds` x U Gets, U at a time)
  for (uint32_t r = 0; r < rounds; ++r) {
  uint64_t key[U], h[U];
  uint32_t seg[U];
  uint8_t s[U];
  bool live[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t op = q0 + ((uint64_t)r * U + (uint64_t)u) * nq;
    live[u] = op < n;
    key[u] = live[u] ? keys[op] : kInvalid;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    h[u] = hash64(key[u]);
    s[u] = 0;
    if (live[u] && reserved_key(key[u])) {
      s[u] = 3;
      live[u] = false;
    } else if (live[u] && wrong_shard(h[u], g.sbits, g.shard)) {
      s[u] = 8;
      live[u] = false;
    }
    seg[u] = live[u] ? de_seg(dir_entry(g, h[u])) : 0u;
  }
  // An even home line is the first half of a 128-B HBM line: the window's
  // second 64-B line comes with it (same request), so it is loaded too and a
  // Get that runs past its home line continues without a dependent round
  // trip.  (Odd home lines: the second line is in the next 128-B line.)
  ulonglong2 p[U], p2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t l0 = (uint32_t)(h[u] & 0xFF);
    const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots + l0 * 4u + q;
    if (live[u]) p[u] = sp[0];
    p2[u] = live[u] && p2on && !(l0 & 1u) ? sp[4] : make_ulonglong2(kInvalid, 0);
  }
  uint64_t val[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    val[u] = 0;
    if (!live[u]) continue;
    const uint32_t mn = (uint32_t)(__ballot(p[u].x == key[u]) >> qbase) & 0xFu;
    const uint32_t en = (uint32_t)(__ballot(p[u].x == kInvalid) >> qbase) & 0xFu;
    const uint32_t line0 = (uint32_t)(h[u] & 0xFF);
    const bool has2 = p2on && !(line0 & 1u);  // the second line was loaded with the first
    uint32_t m1 = 0, e1 = 0;
    if (!mn && !en && has2) {
      m1 = (uint32_t)(__ballot(p2[u].x == key[u]) >> qbase) & 0xFu;
      e1 = (uint32_t)(__ballot(p2[u].x == kInvalid) >> qbase) & 0xFu;
    }
    if (mn) {
      val[u] = shfl64(p[u].y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
      s[u] = 1;
      lines += 1;
    } else if (en) {
      lines += 1;
    } else if (m1) {
      val[u] = shfl64(p2[u].y, (int)(qbase + (uint32_t)__builtin_ctz(m1)));
      s[u] = 1;
      lines += 2;
    } else if (e1) {
      lines += 2;
    } else {
      // rare: continue the window from its second (even home: third) line
      const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots;
      uint32_t t = has2 ? 2 : 1;
      for (; t < kLines; ++t) {
        const ulonglong2 pp = sp[((line0 + t) & 255u) * 4u + q];
        const uint32_t m2 = (uint32_t)(__ballot(pp.x == key[u]) >> qbase) & 0xFu;
        const uint32_t e2 = (uint32_t)(__ballot(pp.x == kInvalid) >> qbase) & 0xFu;
        if (m2) {
          val[u] = shfl64(pp.y, (int)(qbase + (uint32_t)__builtin_ctz(m2)));
          s[u] = 1;
          break;
        }
        if (e2) break;
      }
      lines += (t < kLines ? t + 1 : kLines);
    }
  }
  if (q == 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t op = q0 + ((uint64_t)r * U + (uint64_t)u) * nq;
      if (op < n) {
        if (st) {
          vout[op] = val[u];
          st[op] = s[u];
        } else {  // routing response record
          reinterpret_cast<ulonglong2*>(vout)[op] = make_ulonglong2(val[u], (unsigned long long)s[u]);
        }
      }
    }
  }
  }
  if (COUNT) {
    __shared__ uint32_t red[4];
    uint32_t v = (q == 0) ? lines : 0;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) line_partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

// ------------------------------------------------------------ mixed batches

#ifndef PMDFC_BULK_CLEAR_SHIFT
#define PMDFC_BULK_CLEAR_SHIFT 4  // (A/B builds) the verify pass clears the whole set past (slots >> this) entries
#endif
constexpr uint32_t kBulkClearShift = PMDFC_BULK_CLEAR_SHIFT;
constexpr uint32_t kWrapLine = (kSlots - kWindow) / 4 + 1;  // home lines >= this: the window wraps

// ---- mixed batches, two exact ways to tell a Get whether the batch inserts
// its key (the host picks one per batch, pmdfc_cceh.mixed_join):
//   * the INSERT set (k_mixed_prep + k_mixed_get_iset): every insert of the
//     batch puts its key into a device-wide set (a CAS each), and the Gets that
//     need it probe the set -- cheap when the batch inserts little (config 3:
//     5 % inserts);
//   * the JOIN (k_mixed_get + k_mixed_join, round 6): the Gets that need it
//     claim their keys instead, and every insert looks its key up in that much
//     smaller set -- ~500k random CASes fewer in a half-insert batch (config 4).
// Pre-pass of a mixed batch: hash, reserved key / wrong shard, and the batch's
// set of inserted keys (open addressing, load <= 1/2): the first insert of a
// key stores its batch position, a later one flags the key as inserted more
// than once.  The set is empty on entry (the previous mixed batch's verify
// pass cleared the slots it used, islot); each op's early flag starts at 0,
// and thread 0 opens the batch's drop log.  Each block counts its inserts
// (icount) for the verify pass's choice of how to empty the set.
__global__ __launch_bounds__(256) void k_mixed_prep(const uint8_t* __restrict__ ops,
                                                    const uint64_t* __restrict__ keys,
                                                    uint8_t* __restrict__ st,
                                                    uint64_t* __restrict__ vout, uint64_t n, Geo g,
                                                    uint64_t* __restrict__ iset, uint64_t imask,
                                                    uint32_t* __restrict__ ipos,
                                                    uint32_t* __restrict__ icnt, uint8_t* __restrict__ early,
                                                    uint32_t* __restrict__ islot, DevCtl* __restrict__ ctl,
                                                    uint32_t* __restrict__ loss0, uint32_t* __restrict__ icount) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i == 0) {
    *loss0 = ctl->loss_events;
    ctl->drop_n = 0;  // the batch's drop log starts empty
  }
  __shared__ uint32_t s_ins;
  if (threadIdx.x == 0) s_ins = 0;
  __syncthreads();
  if (i < n) {
  const uint64_t key = keys[i];
  const uint64_t h = hash64(key);
  uint8_t s = kStPending;
  if (reserved_key(key)) s = 3;
  else if (wrong_shard(h, g.sbits, g.shard)) s = 8;
  st[i] = s;
  vout[i] = 0;
  early[i] = 0;
  uint32_t my = 0xFFFFFFFFu;
  const bool ins = s == kStPending && ops[i] == 1;
  if (ins) {
    for (uint64_t sl = iset_slot(h, imask);; sl = (sl + 1) & imask) {
      const uint64_t prev = atomicCAS((unsigned long long*)&iset[sl], (unsigned long long)kInvalid,
                                      (unsigned long long)key);
      if (prev == kInvalid) {  // the only insert of this key so far: its position
        ipos[sl] = (uint32_t)i;
        my = (uint32_t)sl;
        break;
      }
      if (prev == key) {  // inserted more than once in this batch
        icnt[sl] = 1u;
        my = (uint32_t)sl;
        break;
      }
    }
  }
  islot[i] = my;
  const uint64_t b = __ballot(ins);
  if ((threadIdx.x & 63u) == 0 && b) atomicAdd(&s_ins, (uint32_t)__popcll(b));
  }
  __syncthreads();
  if (threadIdx.x == 0) icount[blockIdx.x] = s_ins;  // (k_mixed_get sums them into ctl->ins_total)
}

// Early answers of a mixed batch's Gets, against the pre-batch image.  A Get
// of a key the batch never inserts keeps its pre-batch answer wherever it
// sits in the batch: inserts of other keys only take free slots, and splits
// move entries without changing what a probe returns for a key with one copy.
// A miss stays a miss (nothing adds the key); a single-copy hit keeps its
// value unless a split of this batch drops it (CCEH_hybrid.cpp:24-27,
// split_loss) -- k_mixed_verify checks that.  Keys with several copies (a
// split may reorder them) stay pending.
//   A single-copy hit whose window does not wrap (home line < kWrapLine) is
// answered WITHOUT the inserted-key set (early 3), even if the batch inserts
// the key again: every slot of a window before a stored entry, in probe
// order, is occupied (an entry is placed at the first free slot, by Insert
// and by Split's replay alike, and nothing is ever deleted), so a new copy
// lands after the old one; and a split replays a non-wrapping window in slot
// order = probe order, placing every entry at the first free slot, so two
// copies keep their order (the later one's slot is past the earlier one's)
// and a dropped copy drops every later copy too.  The pre-batch copy stays
// the first copy in probe order -- the reference's Get -- until a split of
// the batch drops it; k_mixed_verify places those drops through the drop log
// (and only then looks at the batch's inserts of the key).  A wrapping window
// (y >= 996) can be replayed out of probe order, and last-writer-wins inserts
// overwrite: those hits probe the set as before.
//   A key the batch inserts exactly once, absent before the batch: if the
// insert comes after this Get the key is still absent (miss now); if before,
// the Get returns that insert's value if it was stored (resolved after the
// batch, kStLinked).  Anything else (copies before the batch, several
// inserts) stays pending, and the batch's ordered bucket passes answer it;
// ctl->pget = tag tells them a Get is left (else the insert-only passes run).
//   A 256-thread block takes 256 consecutive ops: their pending Gets are
// compacted in LDS and its 64 quads take them round-robin, up to kMgU each,
// every quad's key, directory and first window-line loads (and the first
// set slots of the Gets that need the set up front) issued back to back for
// kMgU of them at a time (the inserts cost no quad); a miss that skipped
// the set up front probes it after its window.

template <int kMgU>
__global__ __launch_bounds__(256) void k_mixed_get_iset(const uint8_t* __restrict__ ops,
                                                   const uint64_t* __restrict__ keys,
                                                   uint8_t* __restrict__ st,
                                                   uint64_t* __restrict__ vout, uint64_t n, Geo g,
                                                   const ulonglong2* __restrict__ pairs,
                                                   const uint64_t* __restrict__ iset,
                                                   uint64_t imask, const uint32_t* __restrict__ ipos,
                                                   const uint32_t* __restrict__ icnt,
                                                   uint8_t* __restrict__ early,
                                                   uint32_t* __restrict__ elink, DevCtl* __restrict__ ctl,
                                                   uint32_t tag, uint32_t* __restrict__ icount, uint32_t ups,
                                                   uint32_t* __restrict__ hint_ins) {
  __shared__ uint8_t s_list[256];
  __shared__ uint64_t s_key[256];
  __shared__ uint32_t s_cnt;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t base = (uint64_t)blockIdx.x * 256u;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  {
    // the block's keys are read with its statuses (coalesced, one round trip)
    // and the pending Gets' keys kept in LDS
    const uint64_t i = base + threadIdx.x;
    const bool in = i < n;
    const uint8_t s0 = in ? st[i] : 0, o0 = in ? ops[i] : 1;
    const uint64_t k0 = in ? keys[i] : kInvalid;
    const bool isget = s0 == kStPending && o0 != 1;
    const uint64_t bal = __ballot(isget);
    uint32_t wb = 0;
    if (lane == 0 && bal) wb = atomicAdd(&s_cnt, (uint32_t)__popcll(bal));
    wb = (uint32_t)__shfl((int)wb, 0);
    if (isget) {
      const uint32_t x = wb + (uint32_t)__popcll(bal & ((1ULL << lane) - 1));
      s_list[x] = (uint8_t)threadIdx.x;
      s_key[x] = k0;
    }
  }
  if (blockIdx.x == 0) {  // the batch's inserts, for k_mixed_verify (block-uniform)
    __shared__ uint32_t s_sum[4];
    const uint32_t nblk = (uint32_t)((n + 255) / 256);
    uint32_t c = 0;
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < nblk; j += 256u) c += icount[j];
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_down((int)c, o);
    if (lane == 0) s_sum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
      ctl->ins_total = tot;
      // the batch's inserts for the host's choice of the next batch's mode
      // (a system-scope vector store into coherent pinned memory)
      if (hint_ins) __hip_atomic_store(hint_ins, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  const uint32_t ng = s_cnt;
  const uint32_t quad = threadIdx.x >> 2, q = threadIdx.x & 3u, qbase = lane & ~3u;
  bool pending = false;
  for (uint32_t g0 = 0; g0 < 4u && quad + 64u * g0 < ng; g0 += (uint32_t)kMgU) {
  uint64_t op[kMgU], key[kMgU], h[kMgU], iv[kMgU], iv1[kMgU], sl0[kMgU];
  uint32_t seg[kMgU], ld[kMgU];
  bool live[kMgU], pre[kMgU];
  ulonglong2 p[kMgU], p2[kMgU];
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    const uint32_t idx = quad + 64u * (g0 + (uint32_t)u);
    live[u] = idx < ng;
    op[u] = base + (live[u] ? s_list[idx] : 0u);
    key[u] = live[u] ? s_key[idx] : kInvalid;
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    h[u] = hash64(key[u]);
    const uint32_t e = live[u] ? dir_entry(g, h[u]) : 0u;
    seg[u] = de_seg(e);
    ld[u] = de_ld(e);
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    sl0[u] = iset_slot(h[u], imask);
    const uint32_t l0 = (uint32_t)(h[u] & 0xFF);
    // the set up front only where a hit needs it (a wrapping window, or
    // last-writer-wins); a miss probes it after its window
    pre[u] = live[u] && (ups != 0 || l0 >= kWrapLine);
    iv[u] = pre[u] ? iset[sl0[u]] : kInvalid;
    iv1[u] = pre[u] ? iset[(sl0[u] + 1) & imask] : kInvalid;
    const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots + l0 * 4u + q;
    p[u] = live[u] ? sp[0] : make_ulonglong2(kInvalid, 0);
    // an even home line's 128-B HBM line holds the window's second line too
    // (k_get_u): loaded with it, so the copy count continues without a
    // dependent round trip
    p2[u] = live[u] && !(l0 & 1u) ? sp[4] : make_ulonglong2(kInvalid, 0);
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    if (!live[u]) continue;  // quad-uniform
    // copies of the key in its window (quad_probe_once from the loaded line)
    uint64_t val = 0;
    uint32_t copies = 0;
    {
      const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots;
      const uint32_t line0 = (uint32_t)(h[u] & 0xFF);
      ulonglong2 pp = p[u];
      const ulonglong2 pn = p2[u];
      for (uint32_t t = 0;;) {
        const uint32_t mn = (uint32_t)(__ballot(pp.x == key[u]) >> qbase) & 0xFu;
        const uint32_t en = (uint32_t)(__ballot(pp.x == kInvalid) >> qbase) & 0xFu;
        if (mn && copies == 0) val = shfl64(pp.y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
        copies += (uint32_t)__builtin_popcount(mn);
        if (en || copies > 1 || ++t == kLines) break;
        if (t == 1 && !(line0 & 1u)) pp = pn;
        else pp = sp[((line0 + t) & 255u) * 4u + q];
      }
    }
    const uint8_t c = copies == 0 ? 0 : copies == 1 ? 1 : 2;
    const uint64_t o = op[u];
    if (!pre[u]) {
      if (c == 2) {
        pending = true;
        continue;
      }
      if (c == 1) {  // a non-wrapping single-copy hit: no set (see above)
        if (q == 0) {
          vout[o] = val;
          st[o] = 1;
          early[o] = 3;
        }
        continue;
      }
      iv[u] = iset[sl0[u]];  // a miss: the set after all
      iv1[u] = iset[(sl0[u] + 1) & imask];
    }
    // the batch's inserted-key set (linear probing from the first slot)
    uint64_t sl = ~0ull;
    for (uint64_t s1 = sl0[u], v = iv[u], t = 0;; ++t) {
      if (v == key[u]) {
        sl = s1;
        break;
      }
      if (v == kInvalid) break;
      s1 = (s1 + 1) & imask;
      v = t == 0 ? iv1[u] : iset[s1];
    }
    if (sl != ~0ull) {
      if (c != 0 || icnt[sl] != 0) {
        pending = true;
      } else if (q == 0) {
        const uint32_t ps = ipos[sl];
        if ((uint64_t)ps > o) {
          vout[o] = 0;
          st[o] = 0;
        } else {
          st[o] = kStLinked;
          early[o] = 2;
          elink[o] = ps;
        }
      }
    } else if (c == 2) {
      pending = true;
    } else if (q == 0) {
      vout[o] = c ? val : 0;
      st[o] = c ? 1 : 0;
      early[o] = c;
    }
  }
  }
  if (pending && q == 0) ctl->pget = tag;  // every writer stores the same word
}

// Early answers of a mixed batch's Gets, against the pre-batch image, in the
// batch's first kernel (it also sets every op's status: reserved key, wrong
// shard, pending).  A Get of a key the batch never inserts keeps its
// pre-batch answer wherever it sits in the batch: inserts of other keys only
// take free slots, and splits move entries without changing what a probe
// returns for a key with one copy.  A miss stays a miss (nothing adds the
// key); a single-copy hit keeps its value unless a split of this batch drops
// it (CCEH_hybrid.cpp:24-27, split_loss) -- k_mixed_verify checks that.  Keys
// with several copies (a split may reorder them) stay pending.
//   A single-copy hit whose window does not wrap (home line < kWrapLine) is
// answered whether or not the batch inserts the key again (early 3): every
// slot of a window before a stored entry, in probe order, is occupied (an
// entry is placed at the first free slot, by Insert and by Split's replay
// alike, and nothing is ever deleted), so a new copy lands after the old one;
// and a split replays a non-wrapping window in slot order = probe order,
// placing every entry at the first free slot, so two copies keep their order
// and a dropped copy drops every later copy too.  The pre-batch copy stays the
// first copy in probe order -- the reference's Get -- until a split of the
// batch drops it; k_mixed_verify places those drops through the drop log.
//   The other Gets -- a hit in a wrapping window (a split can replay it out of
// probe order), a hit under last-writer-wins (an insert overwrites), a miss --
// depend on whether the batch inserts their key.  In the JOIN they only mark
// their key's bit in a small filter (one per XCD: kJoinReps replicas, so a
// hot key's marks spread over 8 words; no-return atomics, nothing waits for
// them) and leave their probe result with status kStJoin; k_mixed_join then
// puts into the key set only the inserts whose filter bit is set (the joined
// keys and the filter's false positives: a few thousand CASes per config-4
// batch instead of ~500k), counting them per key with the first position,
// and k_part resolves each kStJoin Get from the set:
//   * no insert of the key: the probe result stands (early 1 for a hit);
//   * a miss whose key the batch inserts exactly once: before the insert a
//     miss, after it linked to the insert (kStLinked, resolved after the batch:
//     the insert's value if it was stored);
//   * anything else: pending, for the batch's ordered bucket passes
//     (ctl->pget = tag: the mixed passes run instead of the insert-only ones).
//   A 256-thread block takes 256 consecutive ops: their pending Gets are
// compacted in LDS and its 64 quads take them round-robin, up to kMgU each,
// every quad's key, directory and first window-line loads issued back to
// back for kMgU of them at a time (the inserts cost no quad).
__device__ __forceinline__ uint32_t jbit_of(uint64_t h) { return (uint32_t)(h >> 24) & (kJoinBits - 1u); }

template <int kMgU>
__global__ __launch_bounds__(256) void k_mixed_get(const uint8_t* __restrict__ ops,
                                                   const uint64_t* __restrict__ keys,
                                                   uint8_t* __restrict__ st,
                                                   uint64_t* __restrict__ vout, uint64_t n, Geo g,
                                                   const ulonglong2* __restrict__ pairs,
                                                   uint8_t* __restrict__ early, uint32_t* __restrict__ islot,
                                                   uint32_t* __restrict__ jbits, DevCtl* __restrict__ ctl,
                                                   uint32_t* __restrict__ loss0, uint32_t tag,
                                                   uint32_t* __restrict__ icount, uint32_t ups) {
  __shared__ uint8_t s_list[256];
  __shared__ uint64_t s_key[256];
  __shared__ uint32_t s_cnt, s_ins;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t base = (uint64_t)blockIdx.x * 256u;
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_ins = 0;
    if (blockIdx.x == 0) {
      *loss0 = ctl->loss_events;
      ctl->drop_n = 0;  // the batch's drop log starts empty
    }
  }
  __syncthreads();
  {
    // every op's status (coalesced), and the pending Gets' keys kept in LDS
    const uint64_t i = base + threadIdx.x;
    const bool in = i < n;
    const uint8_t o0 = in ? ops[i] : 1;
    const uint64_t k0 = in ? keys[i] : kInvalid;
    uint8_t s0 = kStPending;
    if (in) {
      const uint64_t h0 = hash64(k0);
      if (reserved_key(k0)) s0 = 3;
      else if (wrong_shard(h0, g.sbits, g.shard)) s0 = 8;
      st[i] = s0;
      vout[i] = 0;
      early[i] = 0;
      islot[i] = 0xFFFFFFFFu;
    }
    const bool isget = in && s0 == kStPending && o0 != 1;
    const uint64_t bal = __ballot(isget), bins = __ballot(in && s0 == kStPending && o0 == 1);
    uint32_t wb = 0;
    if (lane == 0 && bal) wb = atomicAdd(&s_cnt, (uint32_t)__popcll(bal));
    if (lane == 0 && bins) atomicAdd(&s_ins, (uint32_t)__popcll(bins));
    wb = (uint32_t)__shfl((int)wb, 0);
    if (isget) {
      const uint32_t x = wb + (uint32_t)__popcll(bal & ((1ULL << lane) - 1));
      s_list[x] = (uint8_t)threadIdx.x;
      s_key[x] = k0;
    }
  }
  __syncthreads();
  const uint32_t ng = s_cnt;
  const uint32_t quad = threadIdx.x >> 2, q = threadIdx.x & 3u, qbase = lane & ~3u;
  const uint32_t rep = blockIdx.x & (kJoinReps - 1u);
  bool pending = false, join = false;
  for (uint32_t g0 = 0; g0 < 4u && quad + 64u * g0 < ng; g0 += (uint32_t)kMgU) {
  uint64_t op[kMgU], key[kMgU], h[kMgU];
  uint32_t seg[kMgU];
  bool live[kMgU];
  ulonglong2 p[kMgU], p2[kMgU];
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    const uint32_t idx = quad + 64u * (g0 + (uint32_t)u);
    live[u] = idx < ng;
    op[u] = base + (live[u] ? s_list[idx] : 0u);
    key[u] = live[u] ? s_key[idx] : kInvalid;
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    h[u] = hash64(key[u]);
    seg[u] = live[u] ? de_seg(dir_entry(g, h[u])) : 0u;
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    const uint32_t l0 = (uint32_t)(h[u] & 0xFF);
    const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots + l0 * 4u + q;
    p[u] = live[u] ? sp[0] : make_ulonglong2(kInvalid, 0);
    // an even home line's 128-B HBM line holds the window's second line too
    // (k_get_u): loaded with it, so the copy count continues without a
    // dependent round trip
    p2[u] = live[u] && !(l0 & 1u) ? sp[4] : make_ulonglong2(kInvalid, 0);
  }
#pragma unroll
  for (int u = 0; u < kMgU; ++u) {
    if (!live[u]) continue;  // quad-uniform
    // copies of the key in its window (quad_probe_once from the loaded line)
    uint64_t val = 0;
    uint32_t copies = 0;
    const uint32_t line0 = (uint32_t)(h[u] & 0xFF);
    {
      const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots;
      ulonglong2 pp = p[u];
      const ulonglong2 pn = p2[u];
      for (uint32_t t = 0;;) {
        const uint32_t mn = (uint32_t)(__ballot(pp.x == key[u]) >> qbase) & 0xFu;
        const uint32_t en = (uint32_t)(__ballot(pp.x == kInvalid) >> qbase) & 0xFu;
        if (mn && copies == 0) val = shfl64(pp.y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
        copies += (uint32_t)__builtin_popcount(mn);
        if (en || copies > 1 || ++t == kLines) break;
        if (t == 1 && !(line0 & 1u)) pp = pn;
        else pp = sp[((line0 + t) & 255u) * 4u + q];
      }
    }
    const uint64_t o = op[u];
    if (copies > 1) {  // several copies: the ordered passes (st stays pending)
      pending = true;
      continue;
    }
    if (copies == 1 && !ups && line0 < kWrapLine) {  // a non-wrapping single-copy hit (see above)
      if (q == 0) {
        vout[o] = val;
        st[o] = 1;
        early[o] = 3;
      }
      continue;
    }
    // a joining Get: its probe result, its key's filter bit (no return)
    if (q == 0) {
      vout[o] = copies ? val : 0;
      early[o] = (uint8_t)copies;
      st[o] = kStJoin;
      const uint32_t jb = jbit_of(h[u]);
      atomicOr(&jbits[(size_t)(jb >> 5) * kJoinReps + rep], 1u << (jb & 31u));
    }
    join = true;
  }
  }
  if (pending && q == 0) ctl->pget = tag;  // every writer stores the same word
  if (join && q == 0) ctl->njoin = tag;
  __syncthreads();
  if (threadIdx.x == 0) icount[blockIdx.x] = s_ins;  // (k_mixed_join sums them: the host's mode hint)
}

// The inserts' side of the join (see k_mixed_get): a pending insert whose
// key's bit is set in any filter replica (the 8 words of one bit are
// adjacent: one 32-B load) puts its key into the set, counts itself there and
// keeps the first position (ipos starts at ~0: k_mixed_verify leaves every
// slot it empties that way).  Exits at once when no Get of the batch joined.
// Block 0 sums the batch's inserts for the host (the next batch's mode).
__global__ __launch_bounds__(256) void k_mixed_join(const uint8_t* __restrict__ ops,
                                                    const uint64_t* __restrict__ keys,
                                                    const uint8_t* __restrict__ st, uint64_t n,
                                                    uint64_t* __restrict__ iset, uint64_t imask,
                                                    uint32_t* __restrict__ ipos, uint32_t* __restrict__ icnt,
                                                    uint32_t* __restrict__ islot,
                                                    const uint32_t* __restrict__ jbits, DevCtl* __restrict__ ctl,
                                                    uint32_t tag, const uint32_t* __restrict__ icount,
                                                    uint32_t* __restrict__ hint_ins) {
  static_assert(kJoinReps == 8, "one 32-B filter load per key");
  // the op's loads issued with the control word's (three round trips in all:
  // these, the filter, the set)
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const bool in = i < n;
  const uint8_t o0 = in ? ops[i] : 0, st0 = in ? st[i] : 0;
  const uint64_t key = in ? keys[i] : kInvalid;
  const bool any = ctl->njoin == tag;
  if (blockIdx.x == 0) {
    __shared__ uint32_t s_sum[4];
    const uint32_t nblk = (uint32_t)((n + 255) / 256);
    uint32_t c = 0;
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < nblk; j += 256u) c += icount[j];
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_down((int)c, o);
    if ((threadIdx.x & 63u) == 0) s_sum[threadIdx.x >> 6] = c;
    __syncthreads();
    // the batch's inserts (a system-scope vector store into coherent pinned memory)
    if (threadIdx.x == 0 && hint_ins)
      __hip_atomic_store(hint_ins, s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!any || !in || o0 != 1 || st0 != kStPending) return;
  const uint64_t h = hash64(key);
  const uint32_t jb = jbit_of(h);
  const uint4* fw = reinterpret_cast<const uint4*>(jbits + (size_t)(jb >> 5) * kJoinReps);
  const uint4 f0 = fw[0], f1 = fw[1];
  if (!(((f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w) >> (jb & 31u)) & 1u)) return;
  uint64_t sl = iset_slot(h, imask);
  for (;; sl = (sl + 1) & imask) {
    const uint64_t prev = atomicCAS((unsigned long long*)&iset[sl], (unsigned long long)kInvalid,
                                    (unsigned long long)key);
    if (prev == kInvalid || prev == key) break;
  }
  islot[i] = (uint32_t)sl;
  atomicAdd(&icnt[sl], 1u);
  atomicMin(&ipos[sl], (uint32_t)i);
}

// Upsert batches (PMDFC_CFG_UPSERT): the pre-batch slot of every Insert's key
// in its window (0xFFFF: absent), quad per op, probing to the first empty slot
// like k_get.  The first apply pass takes its UPDATE slots from
// here instead of probing the segment lane by lane; it runs before any split
// of the batch, so these slots are still where the keys are.
__global__ __launch_bounds__(256) void k_upsert_probe(const uint64_t* __restrict__ keys, uint32_t kvs,
                                                      const uint8_t* __restrict__ ops, uint64_t n, Geo g,
                                                      const ulonglong2* __restrict__ pairs,
                                                      uint16_t* __restrict__ upos) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  if (op >= n) return;  // whole quads
  const uint64_t key = keys[op * kvs];
  const uint64_t h = hash64(key);
  const bool live = !reserved_key(key) && (!ops || ops[op] == 1) && !wrong_shard(h, g.sbits, g.shard);
  uint32_t res = 0xFFFFu;
  if (live) {  // quad-uniform
    const ulonglong2* sp = pairs + (size_t)de_seg(dir_entry(g, h)) * kSlots;
    const uint32_t line0 = (uint32_t)(h & 0xFF);
    const uint32_t qbase = (__lane_id() & 63u) & ~3u;
    // a fresh key probes to its window's first empty slot, often several
    // lines: from an even line, the next line is in the same 128-B HBM line
    // and is loaded with it (one round trip per two lines)
    for (uint32_t t = 0; t < kLines;) {
      const uint32_t ln = (line0 + t) & 255u;
      const bool two = !(ln & 1u) && t + 1 < kLines;
      const ulonglong2 p = sp[ln * 4u + q];
      const ulonglong2 pn = two ? sp[ln * 4u + 4u + q] : p;
      const uint32_t mn = (uint32_t)(__ballot(p.x == key) >> qbase) & 0xFu;
      const uint32_t en = (uint32_t)(__ballot(p.x == kInvalid) >> qbase) & 0xFu;
      if (mn) {
        res = ln * 4u + (uint32_t)__builtin_ctz(mn);
        break;
      }
      if (en) break;
      if (two) {
        const uint32_t m2 = (uint32_t)(__ballot(pn.x == key) >> qbase) & 0xFu;
        const uint32_t e2 = (uint32_t)(__ballot(pn.x == kInvalid) >> qbase) & 0xFu;
        if (m2) {
          res = (ln + 1u) * 4u + (uint32_t)__builtin_ctz(m2);
          break;
        }
        if (e2) break;
      }
      t += two ? 2u : 1u;
    }
  }
  if (q == 0) upos[op] = (uint16_t)res;
}

void launch_upsert_probe(const uint64_t* keys, uint32_t kvs, const uint8_t* ops, uint64_t n, Geo g,
                         const ulonglong2* pairs, uint16_t* upos, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_upsert_probe, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, keys, kvs, ops, n, g, pairs,
                       upos);
}

// After a mixed batch: if a split dropped entries during it, re-probe the
// early single-copy hits and the Gets linked to their one insert.  A key
// still stored keeps its answer.  A key that is gone was dropped by a split
// of this batch (Insert4split, CCEH_hybrid.cpp:24-27; the batch never adds it
// back): the drop log holds it with the batch position of the insert whose
// full window caused that split.  In the serial order the drop happens inside
// that insert, so a Get after it misses and a Get before it sees the key --
// the reference's answer either way.  (A key has at most one copy here, so it
// is logged at most once.)  Only a log that overflowed (more than kDropLog
// drops in one batch) leaves the position unknown: PMDFC_ST_SPLIT_LOST and
// the sticky error bit 16.  Linked Gets (early == 2) take their insert's
// outcome first.
//   Early hits answered without the set (early == 3: a non-wrapping window,
// so copies of the key stay in probe order and a split drops a SUFFIX of
// them, see k_mixed_get) stand unless the log holds a drop of the key before
// the Get.  Then the key's copies are replayed as a count: the pre-batch
// copy, + 1 for each stored insert of the key before the Get (a wave scans
// the batch), - 1 for each logged drop, a drop at position t coming before
// the insert at t (that insert's full window split the segment); the Get
// sees the first copy: the pre-batch value while the count never reached 0,
// else the value of the insert that refilled it, or a miss.  (More than 64
// such drops of one key before one Get: PMDFC_ST_SPLIT_LOST, error bit 16.)
__device__ __noinline__ void replay_unchecked_hit(const uint8_t* __restrict__ ops, const uint64_t* __restrict__ keys,
                                                  const uint64_t* __restrict__ vin, uint8_t* __restrict__ st,
                                                  uint64_t* __restrict__ vout, uint64_t o, DevCtl* __restrict__ ctl,
                                                  const ulonglong2* __restrict__ drops) {
  const uint32_t lane = __lane_id() & 63u;
  const uint64_t key = keys[o];
  const uint32_t nd = ctl->drop_n, nl = min(nd, kDropLog);
  // this key's drops before o, one per lane (at most 64)
  uint32_t dtrig = 0xFFFFFFFFu, cnt = 0;
  for (uint32_t j0 = 0; j0 < nl; j0 += 64) {
    const uint32_t j = j0 + lane;
    const ulonglong2 d = j < nl ? drops[j] : make_ulonglong2(kInvalid, 0);
    const bool mine = d.x == key && d.y < o;
    const uint64_t mm = __ballot(mine);
    uint32_t xi = cnt;  // lane xi keeps the xi-th drop
    for (uint64_t b = mm; b; b &= b - 1, ++xi) {
      const uint32_t tv = (uint32_t)__shfl((int)(uint32_t)d.y, __builtin_ctzll(b));
      if (lane == xi) dtrig = tv;
    }
    cnt += (uint32_t)__popcll(mm);
  }
  if (cnt == 0 && nd <= kDropLog) return;  // the pre-batch copy outlived the Get: the early hit stands
  if (nd > kDropLog || cnt > 64u) {        // unplaced
    if (lane == 0) {
      st[o] = 10;  // PMDFC_ST_SPLIT_LOST
      vout[o] = 0;
      atomicOr(&ctl->err, 1u << 16);
    }
    return;
  }
  int len = 1;  // copies of the key, the first one's value
  uint64_t first = vout[o];
  bool applied = lane >= cnt;
  bool bad = false;
  const auto drop_to = [&](uint64_t pos) {  // every drop at or before pos
    const bool now = !applied && dtrig <= pos;
    const int k = (int)__popcll(__ballot(now));
    applied |= now;
    len -= k;
    if (len < 0) {
      bad = true;
      len = 0;
    }
  };
  for (uint64_t p0 = 0; p0 < o; p0 += 64) {
    const uint64_t p = p0 + lane;
    const bool ins = p < o && ops[p] == 1 && keys[p] == key && st[p] == 2;  // a stored insert of the key
    for (uint64_t b = __ballot(ins); b; b &= b - 1) {
      const int src = __builtin_ctzll(b);
      const uint64_t pos = p0 + (uint64_t)src;
      drop_to(pos);
      if (len == 0) first = vin[pos];
      ++len;
    }
  }
  drop_to(o);
  if (lane == 0) {
    st[o] = len > 0 ? 1 : 0;
    vout[o] = len > 0 ? first : 0;
    if (bad) atomicOr(&ctl->err, 4u);  // (cannot happen: more drops than copies)
  }
}

__global__ __launch_bounds__(256) void k_mixed_verify(const uint8_t* __restrict__ ops,
                                                      const uint64_t* __restrict__ keys,
                                                      const uint64_t* __restrict__ vin,
                                                      uint8_t* __restrict__ st,
                                                      uint64_t* __restrict__ vout, uint64_t n, Geo g,
                                                      const ulonglong2* __restrict__ pairs,
                                                      const uint8_t* __restrict__ early,
                                                      const uint32_t* __restrict__ elink,
                                                      DevCtl* __restrict__ ctl,
                                                      const uint32_t* __restrict__ loss0,
                                                      const ulonglong2* __restrict__ drops,
                                                      uint64_t* __restrict__ iset, uint32_t* __restrict__ icnt,
                                                      uint32_t* __restrict__ ipos,
                                                      const uint32_t* __restrict__ islot, uint64_t imask,
                                                      uint32_t* __restrict__ jbits) {  // (null: an insert-set batch)
  // a thread per op; the rare re-probe (a split of this batch dropped
  // entries) is done by the whole wave, one op at a time
  const uint64_t op = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  // the set and the join filter, empty again for the next mixed batch: the
  // slots of this batch's joining Gets (scattered stores), or with many of
  // them the whole set (coalesced stores: 12 B per slot against ~2 scattered
  // stores per key); the filter (1 MiB) whole whenever a Get joined
  // (ipos too, back to ~0: the join's first-position minimum starts there)
  const uint64_t nt = (uint64_t)gridDim.x * 256u;
  if (jbits)
    for (uint64_t x = op; x < kJoinWords; x += nt) jbits[x] = 0u;
  if (!jbits && ctl->ins_total > (uint32_t)((imask + 1) >> kBulkClearShift)) {
    for (uint64_t x = op; x <= imask; x += nt) {
      iset[x] = kInvalid;
      icnt[x] = 0u;
      ipos[x] = 0xFFFFFFFFu;
    }
  } else if (op < n) {
    const uint32_t sl = islot[op];
    if (sl != 0xFFFFFFFFu) {
      iset[sl] = kInvalid;
      icnt[sl] = 0u;
      ipos[sl] = 0xFFFFFFFFu;
    }
  }
  const uint8_t e = op < n ? early[op] : 0;
  bool hit = e == 1;
  const uint64_t m3 = __ballot(e == 3);
  if (e == 2) {
    const uint32_t p = elink[op];
    hit = st[p] == 2 || st[p] == 11;  // PMDFC_ST_INSERTED, PMDFC_ST_UPDATED (upsert)
    vout[op] = hit ? vin[p] : 0;
    st[op] = hit ? 1 : 0;
  }
  uint64_t m = __ballot(hit);
  if ((!m && !m3) || ctl->loss_events == *loss0) return;
  for (uint64_t b = m3; b; b &= b - 1)
    replay_unchecked_hit(ops, keys, vin, st, vout, shfl64(op, __builtin_ctzll(b)), ctl, drops);
  const uint32_t q = lane & 3u;
  while (m) {
    const int src = __builtin_ctzll(m);
    m &= m - 1;
    const uint64_t o = shfl64(op, src);
    const uint64_t key = keys[o];
    const uint64_t h = hash64(key);
    uint64_t val = 0;
    uint32_t lines;
    const uint32_t seg = de_seg(dir_entry(g, h));
    // (every quad probes the same key: a wave-uniform answer)
    if (quad_probe(pairs + (size_t)seg * kSlots, key, h, q, &val, &lines) != 0) continue;
    // gone: find the drop in the log, 64 entries per step
    const uint32_t nd = ctl->drop_n, nl = min(nd, kDropLog);
    uint32_t trig = 0xFFFFFFFFu;
    bool found = false;
    for (uint32_t j0 = 0; j0 < nl && !found; j0 += 64) {
      const uint32_t j = j0 + lane;
      const ulonglong2 d = j < nl ? drops[j] : make_ulonglong2(kInvalid, 0);
      const uint64_t mm = __ballot(d.x == key);
      if (mm) {
        found = true;
        trig = (uint32_t)__shfl((int)(uint32_t)d.y, __builtin_ctzll(mm));
      }
    }
    if (lane != 0) continue;
    if (!found) {
      st[o] = 10;  // PMDFC_ST_SPLIT_LOST (drop log overflowed)
      vout[o] = 0;
      atomicOr(&ctl->err, 1u << 16);
    } else if ((uint64_t)trig < o) {
      st[o] = 0;  // dropped before this Get: the reference misses
      vout[o] = 0;
    }  // else dropped after it: the early hit stands
  }
}

// Fresh table: CCEH(initCap) makes 2^depth segments of local depth `depth`
// (CCEH_hybrid.cpp:79-85).  Bucket b's sub-directory starts at pool offset
// b * 2^db0 with db0 = depth - shard_bits - p1, i.e. the pool begins as the
// flat directory and segment id = directory index.  The same launch zeroes
// the per-bucket words of the passes (z: record cursors, stat slots,
// worklist counts, decline flags, grants, grant shards) and, in block 0, the
// control block with the counters of CCEH(initCap) and the host-mapped
// segment-count hint: one launch per reset instead of eight.
__global__ __launch_bounds__(256) void k_init_segments(ulonglong2* __restrict__ pairs,
                                                       uint32_t* __restrict__ occ,
                                                       uint8_t* __restrict__ ldep,
                                                       uint32_t* __restrict__ pool,
                                                       uint64_t* __restrict__ hdr, uint32_t nseg,
                                                       uint32_t depth, uint32_t p1, uint32_t fixed,
                                                       uint32_t region, InitZero z, DevCtl* __restrict__ ctl,
                                                       uint32_t pool_cur, uint32_t* __restrict__ hint) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t db0 = (uint32_t)__builtin_ctz(nseg) - p1;  // nseg = 2^(depth - sbits)
  if (i < (uint64_t)nseg * kSlots) pairs[i] = make_ulonglong2(kInvalid, 0ULL);
  if (i < (uint64_t)nseg * 32u) occ[i] = 0;
  if (i < nseg) {
    ldep[i] = (uint8_t)depth;
    // bucket b's entries: its fixed slot (cceh_kernels.h kFixedBits) or the pool
    const uint32_t at = fixed ? (uint32_t)(i >> db0) * kFixedSlot + (uint32_t)(i & ((1u << db0) - 1u))
                              : region + (uint32_t)i;
    pool[at] = de_make((uint32_t)i, depth);
  }
  const uint32_t nb = 1u << p1;
  if (i < nb) hdr[i] = hdr_make(fixed ? (uint32_t)i * kFixedSlot : region + ((uint32_t)i << db0), db0);
#pragma unroll
  for (int k = 0; k < kInitZero; ++k)
    if (i < z.n[k]) z.p[k][i] = 0;
  if (blockIdx.x == 0) {
    uint32_t* w = reinterpret_cast<uint32_t*>(ctl);
    for (uint32_t j = threadIdx.x; j < sizeof(DevCtl) / 4; j += 256) w[j] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      ctl->nsegs = nseg;
      ctl->max_ld = depth;
      ctl->pool_cur = pool_cur;
      ctl->depth_count[depth] = nseg;
      if (hint) __hip_atomic_store(hint, nseg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Finer directory buckets (p1 -> p1n bits) once every segment's local depth
// allows it (none spans two new buckets): new bucket w takes the slice of its
// old bucket's sub-directory that its d = p1n - p1 extra hash bits select --
// the same pool entries, nothing moves (the slice has db - d bits, db >= d).
__global__ __launch_bounds__(256) void k_rebucket(const uint64_t* __restrict__ old_hdr, uint64_t* __restrict__ hdr,
                                                  uint32_t p1, uint32_t p1n) {
  const uint32_t w = blockIdx.x * 256u + threadIdx.x;
  if (w >= (1u << p1n)) return;
  const uint32_t d = p1n - p1;
  const uint64_t o = old_hdr[w >> d];
  const uint32_t db = hdr_db(o) - d;
  hdr[w] = hdr_make(hdr_off(o) + ((w & ((1u << d) - 1u)) << db), db);
}

// the smallest local depth over the live segments (ids < ctl->nsegs) -> *out
// (which the caller set to ~0)
__global__ __launch_bounds__(256) void k_min_ldep(const uint8_t* __restrict__ ldep, const DevCtl* __restrict__ ctl,
                                                  uint32_t max_segs, uint32_t* __restrict__ out) {
  const uint32_t n = min(ctl->nsegs, max_segs);
  uint32_t m = 0xFFu;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) m = min(m, (uint32_t)ldep[i]);
  for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63u) == 0) atomicMin(out, m);
}

void launch_min_ldep(const uint8_t* ldep, const DevCtl* ctl, uint32_t max_segs, uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_min_ldep, dim3(64), dim3(256), 0, s, ldep, ctl, max_segs, out);
}

void launch_rebucket(const uint64_t* old_hdr, uint64_t* hdr, uint32_t p1, uint32_t p1n, hipStream_t s) {
  hipLaunchKernelGGL(k_rebucket, dim3(((1u << p1n) + 255) / 256), dim3(256), 0, s, old_hdr, hdr, p1, p1n);
}

// occupied-slot count (CCEH::Utilization numerator, CCEH_hybrid.cpp:412-427)
__global__ __launch_bounds__(256) void k_popcount(const uint32_t* __restrict__ occ, uint64_t nwords,
                                                  unsigned long long* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t c = 0;
  for (; i < nwords; i += (uint64_t)gridDim.x * 256u) c += __popc(occ[i]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

// CCEH::FindAnyway (CCEH_hybrid.cpp:482-496; src/cceh.cpp:457-471): the
// reference walks directory entries 0..capacity-1 and, in each, slots
// 0..1023, returning the first pair whose key matches -- no window, no early
// exit.  Inserts and split replays only ever place a key in the segment its
// hash prefix selects (CCEH_hybrid.cpp:119,54), so the first segment in
// directory order holding the key is that one; inside it the answer is the
// first copy in SLOT order, which differs from Get's probe order when the
// window wraps past slot 1023.  One wave per key: 16 slots per
// lane, one ballot per 64-slot stripe, lowest matching slot wins.
__global__ __launch_bounds__(256) void k_find_anyway(const uint64_t* __restrict__ keys,
                                                     uint64_t* __restrict__ vout, uint8_t* __restrict__ st,
                                                     uint64_t n, Geo g, const ulonglong2* __restrict__ pairs) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (op >= n) return;
  const uint64_t key = keys[op];
  const uint64_t h = hash64(key);
  uint64_t val = 0;
  uint8_t s = 0;  // PMDFC_ST_MISS (NONE)
  if (reserved_key(key)) {
    s = 3;
  } else if (wrong_shard(h, g.sbits, g.shard)) {
    s = 8;
  } else {
    const ulonglong2* sp = pairs + (size_t)de_seg(dir_entry(g, h)) * kSlots;
    ulonglong2 p[kSlots / 64];
#pragma unroll
    for (uint32_t j = 0; j < kSlots / 64; ++j) p[j] = sp[j * 64u + lane];  // stripe j: slots 64j..64j+63
#pragma unroll
    for (uint32_t j = 0; j < kSlots / 64; ++j) {
      const uint64_t m = __ballot(p[j].x == key);
      if (m) {
        val = shfl64(p[j].y, __builtin_ctzll(m));
        s = 1;  // PMDFC_ST_HIT
        break;
      }
    }
  }
  if (lane == 0) {
    vout[op] = val;
    st[op] = s;
  }
}

__global__ __launch_bounds__(256) void k_hash(const uint64_t* __restrict__ keys,
                                              uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = hash64(keys[i]);
}

__global__ __launch_bounds__(256) void k_gen_keys(uint64_t seed, uint64_t start,
                                                  uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t ctr = start + i + (seed << 40);
  uint64_t k = splitmix64(ctr);
  if (k == 0 || k >= kSentinel) k = 0x5555555555555555ULL + ctr;
  out[i] = k;
}

// owner shard of each key (top sbits of h) for the routing sort
__global__ __launch_bounds__(256) void k_owner(const uint64_t* __restrict__ keys, uint64_t n,
                                               uint32_t sbits, uint32_t* __restrict__ owner,
                                               uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  owner[i] = sbits ? (uint32_t)(hash64(keys[i]) >> (64 - sbits)) : 0u;
  idx[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_bounds(const uint32_t* __restrict__ sorted_owner,
                                                uint64_t n, uint32_t ngroups,
                                                uint64_t* __restrict__ starts) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i > n) return;
  const int64_t lo = (i == 0) ? -1 : (int64_t)sorted_owner[i - 1];
  const int64_t hi = (i == n) ? (int64_t)ngroups : (int64_t)sorted_owner[i];
  for (int64_t g = lo + 1; g <= hi && g <= (int64_t)ngroups; ++g) starts[g] = i;
}

// ------------------------------------------------------------------ launchers
#define GRID(n, per) dim3((unsigned)(((n) + (per)-1) / (per)))

// A/B knob: 0 = no speculative second-line load for even home lines
static uint32_t get_p2() {
  static const uint32_t v = [] {
    const char* e = getenv("PMDFC_GET_P2");
    return (e && e[0] == '0') ? 0u : 1u;
  }();
  return v;
}

static int get_unroll() {
  static int u = [] {
    const char* e = getenv("PMDFC_GET_UNROLL");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4) ? v : 2;
  }();
  return u;
}

// ---- flat directory for pure-Get batches (one L2 lookup per Get instead of
// header + sub-directory)
__global__ __launch_bounds__(1024) void k_flat_bits(const uint64_t* __restrict__ hdr, uint32_t nb,
                                                    uint32_t p1, uint32_t max_bits, uint32_t* __restrict__ bits) {
  __shared__ uint32_t s_m[16];
  uint32_t m = 0;
  for (uint32_t b = threadIdx.x; b < nb; b += 1024) m = max(m, hdr_db(hdr[b]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) m = max(m, s_m[w]);
    *bits = p1 + m <= max_bits ? p1 + m : 0xFFu;  // too deep: Gets use hdr/pool
  }
}

__global__ __launch_bounds__(256) void k_flatten(const uint64_t* __restrict__ hdr,
                                                 const uint32_t* __restrict__ pool, uint32_t p1,
                                                 uint32_t* __restrict__ flat, const uint32_t* __restrict__ bits) {
  const uint32_t fb = *bits;
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (fb > kFlatMaxBits || x >= (1u << fb)) return;
  const uint32_t w = p1 ? x >> (fb - p1) : 0u;
  const uint64_t hd = hdr[w];
  const uint32_t db = hdr_db(hd);
  const uint32_t sub = db ? (x >> (fb - p1 - db)) & ((1u << db) - 1u) : 0u;
  flat[x] = pool[hdr_off(hd) + sub];
}

void launch_flatten(const uint64_t* hdr, const uint32_t* pool, uint32_t p1, uint32_t* flat,
                    uint32_t* bits, uint32_t max_bits, hipStream_t s) {
  hipLaunchKernelGGL(k_flat_bits, dim3(1), dim3(1024), 0, s, hdr, 1u << p1, p1, min(max_bits, kFlatMaxBits),
                     bits);
  hipLaunchKernelGGL(k_flatten, dim3((1u << kFlatMaxBits) / 256), dim3(256), 0, s, hdr, pool, p1, flat,
                     (const uint32_t*)bits);
}

static uint64_t get_grid_cap() {
  static const uint64_t v = [] {
    const char* e = getenv("PMDFC_GET_GRID");
    return e ? strtoull(e, nullptr, 0) : 0ull;
  }();
  return v;
}

void launch_get(bool count, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                Geo g, const ulonglong2* pairs, uint32_t* partials, hipStream_t s) {
  if (!n) return;
  const int U = get_unroll();
  if (U > 1) {
    const uint64_t quads = (n + U - 1) / U;
    // a launch of several batches' Gets (pmdfc_cceh_get_batches) caps its
    // grid (PMDFC_GET_GRID blocks, 0: none) and loops
    const uint64_t want = (quads + 63) / 64, cap = count ? 0 : get_grid_cap();  // (COUNT: a partial per block)
    const uint64_t nblk = cap && want > cap ? cap : want;
    const uint32_t rounds = (uint32_t)((want + nblk - 1) / nblk);
    const dim3 grid((unsigned)nblk);
#define LG(UU)                                                                               \
  if (count)                                                                                 \
    hipLaunchKernelGGL((k_get_u<UU, true>), grid, dim3(256), 0, s, keys, vout, st, n, g, pairs, \
                       partials, get_p2(), rounds);                                          \
  else                                                                                       \
    hipLaunchKernelGGL((k_get_u<UU, false>), grid, dim3(256), 0, s, keys, vout, st, n, g, pairs, \
                       partials, get_p2(), rounds);
    if (U == 2) {
      LG(2)
    } else {
      LG(4)
    }
#undef LG
    return;
  }
  if (count)
    hipLaunchKernelGGL(k_get<true>, GRID(n, 64), dim3(256), 0, s, keys, vout, st, n, g, pairs, partials);
  else
    hipLaunchKernelGGL(k_get<false>, GRID(n, 64), dim3(256), 0, s, keys, vout, st, n, g, pairs, partials);
}

void launch_mixed_prep(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                       uint64_t n, Geo g, uint64_t* iset, uint64_t imask, uint32_t* ipos, uint32_t* icnt,
                       uint8_t* early, uint32_t* islot, DevCtl* ctl, uint32_t* loss0, uint32_t* icount,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_mixed_prep, GRID(n ? n : 1, 256), dim3(256), 0, s, ops, keys, st, vout, n, g, iset, imask,
                     ipos, icnt, early, islot, ctl, loss0, icount);
}

// Gets per quad issued together: 2 (configs 4 / 3: U=4 3.91 / 5.76, U=2
// 3.95 / 5.96, U=1 3.97 / 5.94 Gops/s); PMDFC_MG_U overrides (A/B)
static int mg_u() {
  static const int U = [] {
    const char* e = getenv("PMDFC_MG_U");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 4) ? v : 2;
  }();
  return U;
}

void launch_mixed_get_iset(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                           uint64_t n, Geo g, const ulonglong2* pairs, const uint64_t* iset, uint64_t imask,
                           const uint32_t* ipos, const uint32_t* icnt, uint8_t* early, uint32_t* elink, DevCtl* ctl,
                           uint32_t tag, uint32_t* icount, uint32_t ups, uint32_t* hint_ins, hipStream_t s) {
  if (!n) return;
  const int U = mg_u();
#define MG(UU)                                                                                             \
  hipLaunchKernelGGL(k_mixed_get_iset<UU>, GRID(n, 256), dim3(256), 0, s, ops, keys, st, vout, n, g, pairs, iset, \
                     imask, ipos, icnt, early, elink, ctl, tag, icount, ups, hint_ins)
  if (U == 1) MG(1);
  else if (U == 2) MG(2);
  else MG(4);
#undef MG
}

void launch_mixed_get(const uint8_t* ops, const uint64_t* keys, uint8_t* st, uint64_t* vout,
                      uint64_t n, Geo g, const ulonglong2* pairs, uint8_t* early, uint32_t* islot, uint32_t* jbits,
                      DevCtl* ctl, uint32_t* loss0, uint32_t tag, uint32_t* icount, uint32_t ups, hipStream_t s) {
  if (!n) return;
  const int U = mg_u();
#define MG(UU)                                                                                              \
  hipLaunchKernelGGL(k_mixed_get<UU>, GRID(n, 256), dim3(256), 0, s, ops, keys, st, vout, n, g, pairs, early, \
                     islot, jbits, ctl, loss0, tag, icount, ups)
  if (U == 1) MG(1);
  else if (U == 2) MG(2);
  else MG(4);
#undef MG
}

void launch_mixed_join(const uint8_t* ops, const uint64_t* keys, const uint8_t* st, uint64_t n,
                       uint64_t* iset, uint64_t imask, uint32_t* ipos, uint32_t* icnt, uint32_t* islot,
                       const uint32_t* jbits, DevCtl* ctl, uint32_t tag, const uint32_t* icount, uint32_t* hint_ins,
                       hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_mixed_join, GRID(n, 256), dim3(256), 0, s, ops, keys, st, n, iset, imask, ipos, icnt, islot,
                       jbits, ctl, tag, icount, hint_ins);
}

void launch_mixed_verify(const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint8_t* st, uint64_t* vout,
                         uint64_t n, Geo g,
                         const ulonglong2* pairs, const uint8_t* early, const uint32_t* elink, DevCtl* ctl,
                         const uint32_t* loss0, const ulonglong2* drops, uint64_t* iset, uint32_t* icnt,
                         uint32_t* ipos, const uint32_t* islot, uint64_t imask, uint32_t* jbits, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_mixed_verify, GRID(n, 256), dim3(256), 0, s, ops, keys, vin, st, vout, n, g, pairs, early,
                       elink, ctl, loss0, drops, iset, icnt, ipos, islot, imask, jbits);
}

void launch_init_segments(ulonglong2* pairs, uint32_t* occ, uint8_t* ldep, uint32_t* pool,
                          uint64_t* hdr, uint32_t nseg, uint32_t depth, uint32_t p1, uint32_t fixed,
                          uint32_t region, const InitZero& z, DevCtl* ctl, uint32_t pool_cur, uint32_t* hint,
                          hipStream_t s) {
  static_assert(sizeof(DevCtl) % 4 == 0, "DevCtl is zeroed by words");
  uint64_t n = std::max<uint64_t>((uint64_t)nseg * kSlots, 1ULL << p1);
  for (int k = 0; k < kInitZero; ++k) n = std::max<uint64_t>(n, z.n[k]);
  hipLaunchKernelGGL(k_init_segments, GRID(n, 256), dim3(256), 0, s, pairs, occ, ldep, pool, hdr,
                     nseg, depth, p1, fixed, region, z, ctl, pool_cur, hint);
}

void launch_popcount(const uint32_t* occ, uint64_t nwords, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_popcount, dim3(1024), dim3(256), 0, s, occ, nwords, out);
}

void launch_find_anyway(const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n, Geo g,
                        const ulonglong2* pairs, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_find_anyway, GRID(n, 4), dim3(256), 0, s, keys, vout, st, n, g, pairs);
}

void launch_hash(const uint64_t* keys, uint64_t* out, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hash, GRID(n, 256), dim3(256), 0, s, keys, out, n);
}

void launch_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_gen_keys, GRID(n, 256), dim3(256), 0, s, seed, start, out, n);
}

void launch_owner(const uint64_t* keys, uint64_t n, uint32_t sbits, uint32_t* owner, uint32_t* idx,
                  hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_owner, GRID(n, 256), dim3(256), 0, s, keys, n, sbits, owner, idx);
}

void launch_bounds(const uint32_t* sorted_owner, uint64_t n, uint32_t ngroups, uint64_t* starts,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_bounds, GRID(n + 1, 256), dim3(256), 0, s, sorted_owner, n, ngroups, starts);
}

}  // namespace pmdfc
