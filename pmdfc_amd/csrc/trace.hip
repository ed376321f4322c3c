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
//   1. newline positions: hipcub DeviceSelect::If over the byte offsets
//   2. k_trace_parse: lane per line -- tokenise (isspace), parse the fields
//      the reference evaluates (inode and offset on every line, size on W/R)
//      as std::stoull does, record key, op, pages; a malformed line (missing
//      field, no digits, overflow: the reference's UB or uncaught throw) is
//      recorded by its index
//   3. inclusive sum of pages (hipcub DeviceScan)
//   4. k_trace_expand: lane per output op -- binary search of its line,
//      coalesced writes of op and key
//   5. k_trace_info: counts, the cut line and the first malformed line
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "cceh_kernels.h"

namespace pmdfc {

struct IsNewline {
  const char* t;
  __device__ __forceinline__ bool operator()(uint64_t i) const { return t[i] == '\n'; }
};

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

__global__ __launch_bounds__(256) void k_trace_expand(const TraceLine* __restrict__ lines,
                                                      const uint64_t* __restrict__ cum,
                                                      const uint64_t* __restrict__ pages,
                                                      uint64_t nlines, uint64_t nout,
                                                      uint8_t* __restrict__ ops,
                                                      uint64_t* __restrict__ keys) {
  const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (j >= nout) return;
  // first line with cum > j
  uint64_t lo = 0, hi = nlines;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (cum[mid] > j) hi = mid;
    else lo = mid + 1;
  }
  const uint64_t b = j - (cum[lo] - pages[lo]);
  const TraceLine L = lines[lo];
  ops[j] = L.op;
  keys[j] = L.key + 4096ull * b;
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

size_t trace_select_temp_bytes(uint64_t nbytes) {
  size_t tb = 0;
  (void)hipcub::DeviceSelect::If(nullptr, tb, hipcub::CountingInputIterator<uint64_t>(0),
                                 (uint64_t*)nullptr, (uint64_t*)nullptr, nbytes,
                                 IsNewline{nullptr});
  return tb;
}

size_t trace_scan_temp_bytes(uint64_t nlines) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tb, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         nlines);
  return tb;
}

hipError_t launch_trace_newlines(const char* text, uint64_t nbytes, uint64_t* nl, uint64_t* d_nnl,
                                 void* temp, size_t temp_bytes, hipStream_t s) {
  return hipcub::DeviceSelect::If(temp, temp_bytes, hipcub::CountingInputIterator<uint64_t>(0), nl,
                                  d_nnl, nbytes, IsNewline{text}, s);
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
  if (nout)
    hipLaunchKernelGGL(k_trace_expand, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, s,
                       lines, cum, pages, nlines, nout, ops, keys);
}

}  // namespace pmdfc
