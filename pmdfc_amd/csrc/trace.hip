// trace.hip -- replay_KV trace ingestion on the device.
//
// server/replay_KV.cpp:209-247 reads a text trace line by line; each line is
// whitespace-separated fields  seq ts OP inode inode_size offset size
// (:24-31).  key = (inode << 32) + offset; an op starting 'W' becomes
// ceil(size/4096) Inserts, 'R' as many Gets, of key + 4096*b (b = 0, 1, ...);
// any other op adds nothing.  Reading stops after the line that brings the
// op count to numData, and the first numData ops are replayed.
//
// Device pipeline (one host read of the line count):
//   1. newline positions: k_nl_count / tile scan / k_nl_write (two coalesced
//      passes over the text)
//   2. k_trace_parse: lane per line -- tokenise (isspace), parse the fields
//      the reference evaluates (inode and offset on every line, size on W/R)
//      as std::stoull does, record key, op, pages; a malformed line (missing
//      field, no digits, overflow: the reference's UB or uncaught throw) is
//      recorded by its index
//   3. inclusive sum of pages (hipcub DeviceScan)
//   4. k_trace_expand: lane per line writes its pages (a wave per line for
//      lines longer than 64 pages, k_trace_expand_long)
//   5. k_trace_info: counts, the cut line and the first malformed line
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "cceh_kernels.h"

namespace pmdfc {

// Newline positions, two passes over the text (a tile = 256 lanes x 64 B):
// k_nl_count counts each tile's newlines, an exclusive scan over tiles gives
// its first output slot, k_nl_write re-reads the tile and writes positions in
// order (block scan of the per-lane counts).  A lane's 64 bytes come as four
// 16-byte loads; '\n' bytes are found with SWAR zero-byte tests.
constexpr uint32_t kNlTile = 256u * 64u;

__device__ __forceinline__ uint64_t nl_mask64(const char* __restrict__ text, uint64_t base,
                                              uint64_t nbytes, bool aligned) {
  uint64_t m = 0;
  if (aligned && base + 64 <= nbytes) {
    const uint4* p = reinterpret_cast<const uint4*>(text + base);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint4 v = p[r];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t y = w4[w] ^ 0x0A0A0A0Au;
        const uint32_t t = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
        // byte c of this word -> bit 16r + 4w + c
        const uint64_t nib = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
        m |= nib << (16 * r + 4 * w);
      }
    }
  } else {
    for (uint64_t b = base; b < nbytes && b < base + 64; ++b)
      if (text[b] == '\n') m |= 1ull << (b - base);
  }
  return m;
}

__global__ __launch_bounds__(256) void k_nl_count(const char* __restrict__ text, uint64_t nbytes,
                                                  int aligned, uint64_t* __restrict__ tile_cnt) {
  const uint64_t base = (uint64_t)blockIdx.x * kNlTile + (uint64_t)threadIdx.x * 64u;
  const uint32_t c = (uint32_t)__popcll(nl_mask64(text, base, nbytes, aligned));
  typedef hipcub::BlockReduce<uint32_t, 256> BR;
  __shared__ typename BR::TempStorage tmp;
  const uint32_t tot = BR(tmp).Sum(c);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_nl_write(const char* __restrict__ text, uint64_t nbytes,
                                                  int aligned, const uint64_t* __restrict__ tile_cnt,
                                                  const uint64_t* __restrict__ tile_off,
                                                  uint64_t* __restrict__ nl) {
  const uint64_t base = (uint64_t)blockIdx.x * kNlTile + (uint64_t)threadIdx.x * 64u;
  uint64_t m = nl_mask64(text, base, nbytes, aligned);
  const uint32_t c = (uint32_t)__popcll(m);
  typedef hipcub::BlockScan<uint32_t, 256> BS;
  __shared__ typename BS::TempStorage tmp;
  uint32_t ex;
  BS(tmp).ExclusiveSum(c, ex);
  uint64_t o = tile_off[blockIdx.x] - tile_cnt[blockIdx.x] + ex;  // inclusive scan -> tile start
  while (m) {
    nl[o++] = base + (uint64_t)__builtin_ctzll(m);
    m &= m - 1;
  }
}

__device__ __forceinline__ bool c_isspace(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

// std::stoull(token) (base 10): optional sign, at least one digit, trailing
// characters ignored, '-' negates modulo 2^64, overflow throws (-> bad)
__device__ __forceinline__ bool parse_ull(const char* t, uint64_t a, uint64_t b, uint64_t* out) {
  bool neg = false;
  if (a < b && (t[a] == '+' || t[a] == '-')) {
    neg = t[a] == '-';
    ++a;
  }
  if (a >= b || t[a] < '0' || t[a] > '9') return false;
  uint64_t v = 0;
  for (; a < b && t[a] >= '0' && t[a] <= '9'; ++a) {
    const uint64_t d = (uint64_t)(t[a] - '0');
    if (v > (~0ull - d) / 10ull) return false;
    v = v * 10ull + d;
  }
  *out = neg ? (0ull - v) : v;
  return true;
}

__global__ __launch_bounds__(256) void k_trace_parse(const char* __restrict__ text, uint64_t nbytes,
                                                     const uint64_t* __restrict__ nl, uint64_t nnl,
                                                     uint64_t nlines, TraceLine* __restrict__ lines,
                                                     uint64_t* __restrict__ pages,
                                                     unsigned long long* __restrict__ first_bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nlines;
       i += (uint64_t)gridDim.x * 256u) {
    const uint64_t s = i == 0 ? 0 : nl[i - 1] + 1;
    const uint64_t e = i < nnl ? nl[i] : nbytes;
    uint64_t fs[7], fe[7];
    uint32_t nf = 0;
    uint64_t p = s;
    while (p < e && nf < 7) {
      while (p < e && c_isspace(text[p])) ++p;
      if (p >= e) break;
      fs[nf] = p;
      while (p < e && !c_isspace(text[p])) ++p;
      fe[nf] = p;
      ++nf;
    }
    TraceLine L{0, 0, 0};
    uint64_t np = 0;
    bool ok = nf >= 6;
    uint64_t inode = 0, off = 0, size = 0;
    if (ok) ok = parse_ull(text, fs[3], fe[3], &inode) && parse_ull(text, fs[5], fe[5], &off);
    if (ok) {
      const char op = text[fs[2]];
      if (op == 'W' || op == 'R') {
        ok = nf >= 7 && parse_ull(text, fs[6], fe[6], &size);
        if (ok) {
          np = size / 4096 + (size % 4096 ? 1 : 0);
          L.op = op == 'W' ? 1 : 0;  // PMDFC_OP_INSERT / PMDFC_OP_GET
        }
      }
      L.key = (inode << 32) + off;
    }
    if (!ok) {
      np = 0;
      atomicMin(first_bad, (unsigned long long)i);
    }
    lines[i] = L;
    pages[i] = np;
  }
}

// Expansion: a lane per line writes its pages (<= kShortPages; the usual
// case, neighbouring lanes write neighbouring runs); longer lines are left to
// k_trace_expand_long, a wave per line, 64 pages per store step.
constexpr uint64_t kShortPages = 64;

__global__ __launch_bounds__(256) void k_trace_expand(const TraceLine* __restrict__ lines,
                                                      const uint64_t* __restrict__ cum,
                                                      const uint64_t* __restrict__ pages,
                                                      uint64_t nlines, uint64_t nout,
                                                      uint8_t* __restrict__ ops,
                                                      uint64_t* __restrict__ keys) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= nlines) return;
  const uint64_t np = pages[i];
  const uint64_t base = cum[i] - np;
  if (np > kShortPages || base >= nout) return;
  const TraceLine L = lines[i];
  const uint64_t end = min(np, nout - base);
  for (uint64_t b = 0; b < end; ++b) {
    ops[base + b] = (uint8_t)L.op;
    keys[base + b] = L.key + 4096ull * b;
  }
}

__global__ __launch_bounds__(256) void k_trace_expand_long(const TraceLine* __restrict__ lines,
                                                           const uint64_t* __restrict__ cum,
                                                           const uint64_t* __restrict__ pages,
                                                           uint64_t nlines, uint64_t nout,
                                                           uint8_t* __restrict__ ops,
                                                           uint64_t* __restrict__ keys) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * 256u) >> 6;
  for (uint64_t i = w0; i < nlines; i += nw) {
    const uint64_t np = pages[i];
    if (np <= kShortPages) continue;
    const uint64_t base = cum[i] - np;
    if (base >= nout) continue;
    const TraceLine L = lines[i];
    const uint64_t end = min(np, nout - base);
    for (uint64_t b = lane; b < end; b += 64) {
      ops[base + b] = (uint8_t)L.op;
      keys[base + b] = L.key + 4096ull * b;
    }
  }
}

// info: [0] ops produced, [1] lines, [2] total ops of the whole trace, [3] cut
// line (the line whose ops reach num_data; nlines if never), [4] first
// malformed line (~0 if none)
__global__ void k_trace_info(const uint64_t* __restrict__ cum, uint64_t nlines, uint64_t num_data,
                             const unsigned long long* __restrict__ first_bad,
                             uint64_t* __restrict__ info) {
  if (threadIdx.x != 0) return;
  const uint64_t total = nlines ? cum[nlines - 1] : 0;
  uint64_t lo = 0, hi = nlines;  // first line with cum >= num_data
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (cum[mid] >= num_data) hi = mid;
    else lo = mid + 1;
  }
  info[0] = total < num_data ? total : num_data;
  info[1] = nlines;
  info[2] = total;
  info[3] = lo;
  info[4] = *first_bad;
}

uint64_t trace_nl_tiles(uint64_t nbytes) { return (nbytes + kNlTile - 1) / kNlTile; }

size_t trace_scan_temp_bytes(uint64_t nlines) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tb, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         nlines);
  return tb;
}

// tile_cnt / tile_off: trace_nl_tiles(nbytes) entries; the inclusive tile scan
// lands in tile_off, its last entry (the newline count) is copied to *d_nnl
hipError_t launch_trace_newlines(const char* text, uint64_t nbytes, uint64_t* nl, uint64_t* d_nnl,
                                 uint64_t* tile_cnt, uint64_t* tile_off, void* temp,
                                 size_t temp_bytes, hipStream_t s) {
  const uint64_t tiles = trace_nl_tiles(nbytes);
  if (!tiles) return hipSuccess;
  const int aligned = ((uintptr_t)text & 15u) == 0;
  hipLaunchKernelGGL(k_nl_count, dim3((unsigned)tiles), dim3(256), 0, s, text, nbytes, aligned, tile_cnt);
  hipError_t e = hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, tile_cnt, tile_off, tiles, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_nl_write, dim3((unsigned)tiles), dim3(256), 0, s, text, nbytes, aligned,
                     (const uint64_t*)tile_cnt, (const uint64_t*)tile_off, nl);
  return hipMemcpyAsync(d_nnl, tile_off + tiles - 1, 8, hipMemcpyDeviceToDevice, s);
}

hipError_t launch_trace_lines(const char* text, uint64_t nbytes, const uint64_t* nl, uint64_t nnl,
                              uint64_t nlines, TraceLine* lines, uint64_t* pages, uint64_t* cum,
                              unsigned long long* first_bad, uint64_t num_data, uint64_t* info,
                              void* temp, size_t temp_bytes, hipStream_t s) {
  if (nlines) {
    const uint64_t blocks = std::min<uint64_t>((nlines + 255) / 256, 8192);
    hipLaunchKernelGGL(k_trace_parse, dim3((unsigned)blocks), dim3(256), 0, s, text, nbytes, nl,
                       nnl, nlines, lines, pages, first_bad);
    hipError_t e = hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, pages, cum, nlines, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_trace_info, dim3(1), dim3(64), 0, s, cum, nlines, num_data,
                     (const unsigned long long*)first_bad, info);
  return hipGetLastError();
}

void launch_trace_expand(const TraceLine* lines, const uint64_t* cum, const uint64_t* pages,
                         uint64_t nlines, uint64_t nout, uint8_t* ops, uint64_t* keys,
                         hipStream_t s) {
  if (nout && nlines) {
    hipLaunchKernelGGL(k_trace_expand, dim3((unsigned)((nlines + 255) / 256)), dim3(256), 0, s,
                       lines, cum, pages, nlines, nout, ops, keys);
    const uint64_t blocks = std::min<uint64_t>((nlines + 3) / 4, 2048);
    hipLaunchKernelGGL(k_trace_expand_long, dim3((unsigned)blocks), dim3(256), 0, s, lines, cum,
                       pages, nlines, nout, ops, keys);
  }
}

}  // namespace pmdfc
