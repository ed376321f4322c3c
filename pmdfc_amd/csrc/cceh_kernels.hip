// cceh_kernels.hip -- hand-written gfx950 kernels of the batched CCEH engine.
//
// Batch semantics: ops are applied as if run serially in batch
// order on CCEH_hybrid.  Because a segment's contents depend only on the
// subsequence of ops whose hash falls in its key range, each segment's ops are
// processed by ONE lane in batch order (k_process), segments in parallel.  An
// insert that finds its window full stops its segment's run; the segment is
// split by k_split (slot-order replay, CCEH_hybrid.cpp:30-67) and the rest of
// the run is re-routed in the next pass.
#include "cceh_device.h"
#include "cceh_kernels.h"

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
      const uint32_t seg = de_seg(g.dir[dir_index(h, g.gdepth, g.sbits)]);
      s = quad_probe(pairs + (size_t)seg * kSlots, key, h, q, &val, &lines);
    }
    if (q == 0) {
      vout[op] = val;
      st[op] = s;
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
                                               uint32_t* __restrict__ line_partials) {
  const uint64_t nq = (uint64_t)gridDim.x * 64u;
  const uint64_t q0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t qbase = (threadIdx.x & 63u) & ~3u;
  uint64_t key[U], h[U];
  uint32_t seg[U];
  uint8_t s[U];
  bool live[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t op = q0 + (uint64_t)u * nq;
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
    seg[u] = live[u] ? de_seg(g.dir[dir_index(h[u], g.gdepth, g.sbits)]) : 0u;
  }
  ulonglong2 p[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (live[u]) p[u] = pairs[(size_t)seg[u] * kSlots + (uint32_t)(h[u] & 0xFF) * 4u + q];
  uint64_t val[U];
  uint32_t lines = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    val[u] = 0;
    if (!live[u]) continue;
    const uint32_t mn = (uint32_t)(__ballot(p[u].x == key[u]) >> qbase) & 0xFu;
    const uint32_t en = (uint32_t)(__ballot(p[u].x == kInvalid) >> qbase) & 0xFu;
    if (mn) {
      val[u] = shfl64(p[u].y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
      s[u] = 1;
      lines += 1;
    } else if (en) {
      lines += 1;
    } else {
      // rare: continue the window from its second line
      const ulonglong2* sp = pairs + (size_t)seg[u] * kSlots;
      const uint32_t line0 = (uint32_t)(h[u] & 0xFF);
      uint32_t t = 1;
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
      const uint64_t op = q0 + (uint64_t)u * nq;
      if (op < n) {
        vout[op] = val[u];
        st[op] = s[u];
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

// --------------------------------------------------------- insert/mixed prep
// hash every op once; resolve reserved keys / wrong shard; mark the rest pending
__global__ __launch_bounds__(256) void k_prep(const uint64_t* __restrict__ keys,
                                              uint64_t* __restrict__ hbuf,
                                              uint8_t* __restrict__ st,
                                              uint64_t* __restrict__ vout, uint64_t n,
                                              uint32_t sbits, uint32_t shard) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  const uint64_t h = hash64(key);
  hbuf[i] = h;
  uint8_t s = kStPending;
  if (reserved_key(key)) s = 3;
  else if (wrong_shard(h, sbits, shard)) s = 8;
  st[i] = s;
  if (vout) vout[i] = 0;
}

// mixed: mark segments that receive an insert in this batch
__global__ __launch_bounds__(256) void k_mark(const uint8_t* __restrict__ ops,
                                              const uint64_t* __restrict__ hbuf,
                                              const uint8_t* __restrict__ st, uint64_t n, Geo g,
                                              uint8_t* __restrict__ touched) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if (ops[i] != 1 || st[i] != kStPending) return;
  touched[de_seg(g.dir[dir_index(hbuf[i], g.gdepth, g.sbits)])] = 1;
}

// mixed: Gets on segments no insert of this batch touches see the pre-batch
// state, so they are answered immediately; everything else becomes pending.
__global__ __launch_bounds__(256) void k_mixed_get(const uint8_t* __restrict__ ops,
                                                   const uint64_t* __restrict__ keys,
                                                   const uint64_t* __restrict__ hbuf,
                                                   uint8_t* __restrict__ st,
                                                   uint64_t* __restrict__ vout, uint64_t n, Geo g,
                                                   const ulonglong2* __restrict__ pairs,
                                                   const uint8_t* __restrict__ touched,
                                                   uint8_t* __restrict__ pend_flag) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  if (op >= n) return;
  uint8_t flag = 0;
  if (st[op] == kStPending) {
    if (ops[op] == 1) {
      flag = 1;
    } else {
      const uint64_t h = hbuf[op];
      const uint32_t seg = de_seg(g.dir[dir_index(h, g.gdepth, g.sbits)]);
      if (touched[seg]) {
        flag = 1;
      } else {
        uint64_t val = 0;
        uint32_t lines;
        const uint8_t s = quad_probe(pairs + (size_t)seg * kSlots, keys[op], h, q, &val, &lines);
        if (q == 0) {
          vout[op] = val;
          st[op] = s;
        }
      }
    }
  }
  if (q == 0) pend_flag[op] = flag;
}

// ------------------------------------------------------------------- route
// sort key = segment id of each pending op (SENT for resolved ops)
__global__ __launch_bounds__(256) void k_route(const uint32_t* __restrict__ pend, uint64_t npend,
                                               const uint64_t* __restrict__ hbuf,
                                               const uint8_t* __restrict__ st, Geo g,
                                               uint32_t sent, uint32_t* __restrict__ skey,
                                               uint32_t* __restrict__ sval) {
  const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (p >= npend) return;
  const uint32_t op = pend ? pend[p] : (uint32_t)p;
  uint32_t seg = sent;
  if (st[op] == kStPending) seg = de_seg(g.dir[dir_index(hbuf[op], g.gdepth, g.sbits)]);
  skey[p] = seg;
  sval[p] = op;
}

// ----------------------------------------------------------------- process
// One 64-lane wave per 64 sorted positions.  The wave gathers its positions'
// op records into LDS cooperatively; every lane that starts a segment run then
// applies that run's ops sequentially, in batch order, against the segment's
// occupancy bitmap held in LDS.  Inserts claim the first free slot of the
// 32-slot window (CCEH_hybrid.cpp:143-168); Gets probe the segment in HBM,
// which already holds this lane's earlier inserts (same-lane program order).
// On a full window the run stops: the segment is queued for k_split and the
// remaining ops of the run are deferred to the next pass.
__global__ __launch_bounds__(64) void k_process(
    const uint32_t* __restrict__ skey, const uint32_t* __restrict__ sval, uint64_t npend,
    uint32_t sent, const uint8_t* __restrict__ ops, const uint64_t* __restrict__ keys,
    const uint64_t* __restrict__ vin, uint64_t* __restrict__ vout, uint8_t* __restrict__ st,
    const uint64_t* __restrict__ hbuf, ulonglong2* __restrict__ pairs,
    uint32_t* __restrict__ occ, const uint8_t* __restrict__ ldep,
    uint8_t* __restrict__ deferred, uint32_t* __restrict__ split_list,
    DevCtl* __restrict__ ctl, uint32_t gdepth, uint32_t max_segments) {
  __shared__ uint32_t s_bm[64][33];
  __shared__ uint64_t s_key[64], s_h[64], s_val[64];
  __shared__ uint32_t s_op[64], s_seg[64];
  __shared__ uint8_t s_code[64];

  const uint32_t lane = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * 64u;
  const uint64_t p0 = base + lane;
  uint32_t seg = sent;
  uint32_t prev = sent;
  if (p0 < npend) {
    seg = skey[p0];
    if (p0 > 0) prev = skey[p0 - 1];
    s_seg[lane] = seg;
    if (seg != sent) {
      const uint32_t op = sval[p0];
      s_op[lane] = op;
      s_key[lane] = keys[op];
      s_h[lane] = hbuf[op];
      const uint8_t code = ops ? ops[op] : (uint8_t)1;
      s_code[lane] = code;
      s_val[lane] = (code == 1 && vin) ? vin[op] : 0;
    }
  }
  const bool start = seg != sent && (p0 == 0 || prev != seg);
  uint32_t* bm = s_bm[lane];
  if (start) {
    const uint4* o = reinterpret_cast<const uint4*>(occ + (size_t)seg * 32u);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 v = o[j];
      bm[4 * j + 0] = v.x;
      bm[4 * j + 1] = v.y;
      bm[4 * j + 2] = v.z;
      bm[4 * j + 3] = v.w;
    }
  }
  __syncthreads();
  if (!start) return;

  ulonglong2* sp = pairs + (size_t)seg * kSlots;
  const uint32_t L = ldep[seg];
  bool dirty = false;
  for (uint64_t p = p0; p < npend; ++p) {
    uint32_t op;
    uint64_t key, h, v;
    uint8_t code;
    if (p < base + 64) {
      const uint32_t i = (uint32_t)(p - base);
      if (s_seg[i] != seg) break;  // run ends inside the tile
      op = s_op[i];
      key = s_key[i];
      h = s_h[i];
      v = s_val[i];
      code = s_code[i];
    } else {
      if (skey[p] != seg) break;
      op = sval[p];
      key = keys[op];
      h = hbuf[op];
      code = ops ? ops[op] : (uint8_t)1;
      v = (code == 1 && vin) ? vin[op] : 0;
    }
    if (code == 1) {
      const uint32_t w = (uint32_t)(h & 0xFF) * 4u;
      const uint32_t wi = w >> 5;
      const int pos = window_first_free(bm[wi], bm[(wi + 1) & 31u], w);
      if (pos < 0) {
        // window full.  The reference would split forever if all 32 entries
        // carry this key's full hash: report UNSPLITTABLE.
        bool same = true;
        for (uint32_t i = 0; i < kWindow && same; ++i)
          same = hash64(sp[(w + i) & (kSlots - 1)].x) == h;
        if (same) {
          st[op] = 4;  // PMDFC_ST_UNSPLITTABLE
          continue;
        }
        if (L + 1 > kMaxDepth) {
          st[op] = 5;  // PMDFC_ST_DEPTH_LIMIT
          continue;
        }
        const uint32_t c1 = atomicAdd(&ctl->nsegs, 1u);
        if (c1 >= max_segments) {
          st[op] = 6;  // PMDFC_ST_CAPACITY
          continue;
        }
        const uint32_t si = atomicAdd(&ctl->n_split, 1u);
        split_list[2 * si] = seg;
        split_list[2 * si + 1] = c1;
        if (L >= gdepth) atomicOr(&ctl->need_double, 1u);
        uint32_t cnt = 0;
        for (uint64_t r = p; r < npend; ++r) {
          if (skey[r] != seg) break;
          deferred[sval[r]] = 1;
          ++cnt;
        }
        atomicAdd(&ctl->n_deferred, cnt);
        break;
      }
      bm[(uint32_t)pos >> 5] |= 1u << ((uint32_t)pos & 31u);
      dirty = true;
      sp[pos] = make_ulonglong2(key, v);
      st[op] = 2;  // PMDFC_ST_INSERTED
    } else {
      uint64_t val = 0;
      const uint8_t s = lane_probe(sp, key, h, &val);
      if (vout) vout[op] = val;
      st[op] = s;
    }
  }
  if (dirty) {
    uint4* o = reinterpret_cast<uint4*>(occ + (size_t)seg * 32u);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = make_uint4(bm[4 * j + 0], bm[4 * j + 1], bm[4 * j + 2], bm[4 * j + 3]);
  }
}

// ------------------------------------------------------------------- split
// Segment::Split, non-INPLACE (CCEH_hybrid.cpp:47-66) + directory update
// (:243-286).  One wave per queued segment.  Child 0 overwrites the parent's
// storage, child 1 goes to the id reserved by k_process.  The replay walks the
// parent in slot order 0..1023 (Insert4split, :18-28): each entry takes the
// first free slot of its own window in its child, or is dropped (split_loss).
// The walk is a wave-uniform scalar loop over readlane'd slot descriptors; the
// two children's bitmaps live in one VGPR (lanes 0-31 child 0, 32-63 child 1).
__global__ __launch_bounds__(64) void k_split(const uint32_t* __restrict__ split_list,
                                              ulonglong2* __restrict__ pairs,
                                              uint32_t* __restrict__ occ,
                                              uint8_t* __restrict__ ldep,
                                              uint32_t* __restrict__ dir, uint32_t gdepth,
                                              uint32_t sbits, DevCtl* __restrict__ ctl) {
  __shared__ ulonglong2 s_par[kSlots];
  __shared__ uint16_t s_inv[2][kSlots];

  const uint32_t lane = threadIdx.x;
  const uint32_t seg = split_list[2 * blockIdx.x];
  const uint32_t c1 = split_list[2 * blockIdx.x + 1];
  const uint32_t L = ldep[seg];
  ulonglong2* sp = pairs + (size_t)seg * kSlots;

  uint32_t inf[16];
  uint64_t any_h = 0;
  bool have = false;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t slot = (uint32_t)j * 64u + lane;
    const ulonglong2 p = sp[slot];
    s_par[slot] = p;
    s_inv[0][slot] = 0;
    s_inv[1][slot] = 0;
    const bool valid = p.x != kInvalid;
    const uint64_t kh = hash64(p.x);
    if (valid && !have) {
      have = true;
      any_h = kh;
    }
    // bit 31: valid, bit 8: child (hash bit 63-L, CCEH_hybrid.cpp:52-55), bits 0-7: home line
    inf[j] = (valid ? 0x80000000u : 0u) | ((uint32_t)((kh >> (63 - L)) & 1u) << 8) |
             (uint32_t)(kh & 0xFF);
  }

  uint32_t b = 0;  // lane l<32: child-0 word l; lane 32+l: child-1 word l
  uint32_t loss = 0;
  uint32_t dest[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t d = 0xFFFFFFFFu;
    uint64_t vm = __ballot((inf[j] & 0x80000000u) != 0);
    while (vm) {
      const int l = __builtin_ctzll(vm);
      vm &= vm - 1;
      const uint32_t si = (uint32_t)__builtin_amdgcn_readlane((int)inf[j], l);
      const uint32_t c = (si >> 8) & 1u;
      const uint32_t w = (si & 0xFFu) * 4u;
      const uint32_t wi = w >> 5;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)(c * 32u + wi));
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)(c * 32u + ((wi + 1u) & 31u)));
      const int pos = window_first_free(lo, hi, w);
      if (pos < 0) {
        ++loss;
        continue;
      }
      const uint32_t wsel = (uint32_t)pos >> 5;
      const uint32_t cur = (wsel == wi) ? lo : hi;
      const uint32_t nw = cur | (1u << ((uint32_t)pos & 31u));
      b = (lane == c * 32u + wsel) ? nw : b;
      d = (lane == (uint32_t)l) ? ((c << 10) | (uint32_t)pos) : d;
    }
    dest[j] = d;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t d = dest[j];
    if (d != 0xFFFFFFFFu) s_inv[d >> 10][d & 1023u] = (uint16_t)(j * 64 + lane + 1);
  }
  __syncthreads();

  // write both children whole (every slot exactly once, coalesced)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    ulonglong2* dst = pairs + (size_t)(c ? c1 : seg) * kSlots;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const uint32_t slot = (uint32_t)j * 64u + lane;
      const uint32_t src = s_inv[c][slot];
      dst[slot] = src ? s_par[src - 1] : make_ulonglong2(kInvalid, 0ULL);
    }
  }
  if (lane < 32) occ[(size_t)seg * 32u + lane] = b;
  else occ[(size_t)c1 * 32u + (lane - 32)] = b;
  if (lane == 0) {
    ldep[seg] = (uint8_t)(L + 1);
    ldep[c1] = (uint8_t)(L + 1);
    atomicMax(&ctl->max_ld, L + 1);
    atomicAdd((unsigned long long*)&ctl->splits, 1ULL);
    if (loss) atomicAdd((unsigned long long*)&ctl->split_loss, (unsigned long long)loss);
  }
  // directory: the 2^(D-L) entries that pointed at the parent; first half
  // keeps child 0 (= parent id), second half gets child 1
  const uint64_t vmask = __ballot(have);
  const int src = vmask ? __builtin_ctzll(vmask) : 0;
  const uint64_t h0 = shfl64(any_h, src);
  const uint32_t Ll = L - sbits;
  const uint32_t Dl = gdepth - sbits;
  const uint64_t prefix = Ll ? ((h0 >> (64 - L)) & ((1ULL << Ll) - 1)) : 0;
  const uint64_t stride = 1ULL << (Dl - Ll);
  const uint64_t xbase = prefix << (Dl - Ll);
  for (uint64_t i = lane; i < stride; i += 64)
    dir[xbase + i] = de_make(i < stride / 2 ? seg : c1, L + 1);
}

// directory doubling (CCEH_hybrid.cpp:208-219): new[2i] = new[2i+1] = old[i]
__global__ __launch_bounds__(256) void k_double(const uint32_t* __restrict__ od,
                                                uint32_t* __restrict__ nd, uint64_t n_new) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n_new) nd[i] = od[i >> 1];
}

__global__ __launch_bounds__(256) void k_init_segments(ulonglong2* __restrict__ pairs,
                                                       uint32_t* __restrict__ occ,
                                                       uint8_t* __restrict__ ldep,
                                                       uint32_t* __restrict__ dir, uint32_t nseg,
                                                       uint32_t depth) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < (uint64_t)nseg * kSlots) pairs[i] = make_ulonglong2(kInvalid, 0ULL);
  if (i < (uint64_t)nseg * 32u) occ[i] = 0;
  if (i < nseg) {
    ldep[i] = (uint8_t)depth;
    dir[i] = de_make((uint32_t)i, depth);
  }
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

static int get_unroll() {
  static int u = [] {
    const char* e = getenv("PMDFC_GET_UNROLL");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4) ? v : 2;
  }();
  return u;
}

void launch_get(bool count, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                Geo g, const ulonglong2* pairs, uint32_t* partials, hipStream_t s) {
  if (!n) return;
  const int U = get_unroll();
  if (U > 1) {
    const uint64_t quads = (n + U - 1) / U;
    const dim3 grid((unsigned)((quads + 63) / 64));
#define LG(UU)                                                                               \
  if (count)                                                                                 \
    hipLaunchKernelGGL((k_get_u<UU, true>), grid, dim3(256), 0, s, keys, vout, st, n, g, pairs, \
                       partials);                                                            \
  else                                                                                       \
    hipLaunchKernelGGL((k_get_u<UU, false>), grid, dim3(256), 0, s, keys, vout, st, n, g, pairs, \
                       partials);
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

void launch_prep(const uint64_t* keys, uint64_t* hbuf, uint8_t* st, uint64_t* vout, uint64_t n,
                 uint32_t sbits, uint32_t shard, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_prep, GRID(n, 256), dim3(256), 0, s, keys, hbuf, st, vout, n, sbits, shard);
}

void launch_mark(const uint8_t* ops, const uint64_t* hbuf, const uint8_t* st, uint64_t n, Geo g,
                 uint8_t* touched, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_mark, GRID(n, 256), dim3(256), 0, s, ops, hbuf, st, n, g, touched);
}

void launch_mixed_get(const uint8_t* ops, const uint64_t* keys, const uint64_t* hbuf, uint8_t* st,
                      uint64_t* vout, uint64_t n, Geo g, const ulonglong2* pairs,
                      const uint8_t* touched, uint8_t* pend_flag, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_mixed_get, GRID(n, 64), dim3(256), 0, s, ops, keys, hbuf, st, vout, n, g,
                       pairs, touched, pend_flag);
}

void launch_route(const uint32_t* pend, uint64_t npend, const uint64_t* hbuf, const uint8_t* st,
                  Geo g, uint32_t sent, uint32_t* skey, uint32_t* sval, hipStream_t s) {
  if (npend)
    hipLaunchKernelGGL(k_route, GRID(npend, 256), dim3(256), 0, s, pend, npend, hbuf, st, g, sent,
                       skey, sval);
}

void launch_process(const uint32_t* skey, const uint32_t* sval, uint64_t npend, uint32_t sent,
                    const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint64_t* vout,
                    uint8_t* st, const uint64_t* hbuf, ulonglong2* pairs, uint32_t* occ,
                    const uint8_t* ldep, uint8_t* deferred, uint32_t* split_list, DevCtl* ctl,
                    uint32_t gdepth, uint32_t max_segments, hipStream_t s) {
  if (npend)
    hipLaunchKernelGGL(k_process, GRID(npend, 64), dim3(64), 0, s, skey, sval, npend, sent, ops,
                       keys, vin, vout, st, hbuf, pairs, occ, ldep, deferred, split_list, ctl,
                       gdepth, max_segments);
}

void launch_split(uint32_t nsplit, const uint32_t* split_list, ulonglong2* pairs, uint32_t* occ,
                  uint8_t* ldep, uint32_t* dir, uint32_t gdepth, uint32_t sbits, DevCtl* ctl,
                  hipStream_t s) {
  if (nsplit)
    hipLaunchKernelGGL(k_split, dim3(nsplit), dim3(64), 0, s, split_list, pairs, occ, ldep, dir,
                       gdepth, sbits, ctl);
}

void launch_double(const uint32_t* od, uint32_t* nd, uint64_t n_new, hipStream_t s) {
  hipLaunchKernelGGL(k_double, GRID(n_new, 256), dim3(256), 0, s, od, nd, n_new);
}

void launch_init_segments(ulonglong2* pairs, uint32_t* occ, uint8_t* ldep, uint32_t* dir,
                          uint32_t nseg, uint32_t depth, hipStream_t s) {
  const uint64_t n = (uint64_t)nseg * kSlots;
  hipLaunchKernelGGL(k_init_segments, GRID(n, 256), dim3(256), 0, s, pairs, occ, ldep, dir, nseg, depth);
}

void launch_popcount(const uint32_t* occ, uint64_t nwords, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_popcount, dim3(1024), dim3(256), 0, s, occ, nwords, out);
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
