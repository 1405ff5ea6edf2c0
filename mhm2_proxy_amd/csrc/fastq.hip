// FASTQ text -> PackedRead bytes on the device ("ingest to the device stream").
//
// Reference: FastqReader::get_next_fq_record (src/fastq.cpp:504-551: four fgets lines per record, rtrim,
// '@' / '+' checks, get_fq_name :73-122, equal sequence and quality lengths) feeding the PackedRead
// constructor (src/packed_reads.cpp:73-109: A0 C1 G2 T3, N and the IUPAC codes U R Y K M S W B D H V -> 4,
// anything else fatal; quality min(q - qual_offset, 31) in bits 3-7).
//
// The text is HBM-resident; the pass is byte streaming:
//   k_fq_count    newlines per 4 KB chunk (16 bytes per lane, SWAR zero-byte test)
//   scan          chunk bases (rocPRIM)
//   k_fq_lines    every newline, in order (block scan of the lanes' counts), as one word: position,
//                 trailing whitespace of the line, first character of the next line
//   k_fq_records  one lane per 4-line record: format checks and sequence length from the line words
//   scan          read offsets (rocPRIM) = the PackedReads CSR layout k_extract_scatter consumes
//   k_fq_pack     one 16-lane group per record: base code | quality << 3
// Errors are reported as the first failing record (atomicMin of record << 4 | kind, kinds as in
// kcount_launch.hpp FQ_E_*), which is where the reference DIEs.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include "kcount_launch.hpp"

namespace mhm {

namespace {

constexpr int FQ_THREADS = 256;
constexpr int FQ_BYTES = 16;  // per lane
static_assert(FQ_THREADS * FQ_BYTES == FQ_CHUNK, "chunk = one block");

// 4-bit mask of the '\n' bytes of a little-endian word (exact zero-byte test of w ^ 0x0a0a0a0a)
__device__ __forceinline__ uint32_t nl4(uint32_t w) {
  const uint32_t x = w ^ 0x0a0a0a0au;
  const uint32_t hi = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
  return ((hi >> 7) & 1u) | ((hi >> 14) & 2u) | ((hi >> 21) & 4u) | ((hi >> 28) & 8u);
}

// 16-bit mask of the newlines among text[pos, pos + 16) (bytes at or past n never match)
__device__ __forceinline__ uint32_t nl_mask(const char *text, uint64_t pos, uint64_t n) {
  if (pos + FQ_BYTES <= n && (((uintptr_t)(text + pos)) & 15u) == 0) {
    const uint4 v = *(const uint4 *)(text + pos);
    return nl4(v.x) | (nl4(v.y) << 4) | (nl4(v.z) << 8) | (nl4(v.w) << 12);
  }
  uint32_t m = 0;
  for (int i = 0; i < FQ_BYTES; i++)
    if (pos + i < n && text[pos + i] == '\n') m |= 1u << i;
  return m;
}

__global__ __launch_bounds__(FQ_THREADS) void k_fq_count(const char *text, uint64_t n, unsigned long long *chunk) {
  __shared__ uint32_t s_w[FQ_THREADS / 64];
  const uint64_t pos = (uint64_t)blockIdx.x * FQ_CHUNK + (uint64_t)threadIdx.x * FQ_BYTES;
  uint32_t c = __popc(nl_mask(text, pos, n));
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < FQ_THREADS / 64; w++) t += s_w[w];
    chunk[blockIdx.x] = t;
  }
}

__device__ __forceinline__ bool fq_space(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// 16 bytes of text from pos (zero past n), with the newline mask
__device__ __forceinline__ uint32_t load16(const char *text, uint64_t pos, uint64_t n, uint32_t (&v)[4]) {
  if (pos + FQ_BYTES <= n && (((uintptr_t)(text + pos)) & 15u) == 0) {
    const uint4 q = *(const uint4 *)(text + pos);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (pos + 4 * i + j < n) x |= (uint32_t)(unsigned char)text[pos + 4 * i + j] << (8 * j);
      v[i] = x;
    }
  }
  uint32_t m = nl4(v[0]) | (nl4(v[1]) << 4) | (nl4(v[2]) << 8) | (nl4(v[3]) << 12);
  if (pos + FQ_BYTES > n) m &= n > pos ? (1u << (n - pos)) - 1u : 0u;  // zero bytes past n are not newlines
  return m;
}
__device__ __forceinline__ unsigned char byte_of(const uint32_t (&v)[4], int i) {
  return (unsigned char)(v[i >> 2] >> (8 * (i & 3)));
}

// Per newline (line j ends at it), one word: its position (bits 0-39), the number of trailing whitespace
// characters of line j (rtrim, src/fastq.cpp:67-71; bits 40-55) and the first character of line j + 1 (the
// newline itself when that line is empty, 0 at the end of the text; bits 56-63). k_fq_records checks
// records from these words instead of re-reading the text for them.
__global__ __launch_bounds__(FQ_THREADS) void k_fq_lines(const char *text, uint64_t n,
                                                          const unsigned long long *chunk_base,
                                                          unsigned long long *line_end) {
  __shared__ uint32_t s_w[FQ_THREADS / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t pos = (uint64_t)blockIdx.x * FQ_CHUNK + (uint64_t)threadIdx.x * FQ_BYTES;
  uint32_t v[4];
  uint32_t m = load16(text, pos, n, v);
  const uint32_t c = __popc(m);
  uint32_t incl = c;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint64_t o = chunk_base[blockIdx.x] + (incl - c);
  for (int w = 0; w < wid; w++) o += s_w[w];
  // the neighbouring lanes' edge bytes (the byte before this lane's 16 and the byte after them), so that
  // only the wave's edge lanes go to memory for them
  const uint32_t prev_w = __shfl_up(v[3], 1, 64), next_w = __shfl_down(v[0], 1, 64);
  while (m) {
    const int b = __ffs(m) - 1;
    m &= m - 1;
    const uint64_t p = pos + (uint64_t)b;
    const unsigned nf = b < FQ_BYTES - 1 ? byte_of(v, b + 1)
                    : lane < 63       ? (unsigned char)next_w
                                      : (p + 1 < n ? (unsigned char)text[p + 1] : 0);
    // trailing whitespace of the line that ends at p: back from p - 1 to the previous newline or the start
    uint32_t t = 0;
    int64_t q = (int64_t)p - 1;
    while (q >= 0 && t < 0xffffu) {
      const unsigned char ch = q >= (int64_t)pos                      ? byte_of(v, (int)(q - (int64_t)pos))
                               : (q == (int64_t)pos - 1 && lane > 0) ? (unsigned char)(prev_w >> 24)
                                                                      : (unsigned char)text[q];
      if (ch == '\n' || !fq_space(ch)) break;
      t++;
      q--;
    }
    line_end[o] = p | ((uint64_t)t << FQ_LE_BITS) | ((uint64_t)nf << 56);
    o++;
  }
}

__device__ __forceinline__ uint64_t rtrim_end(const char *s, uint64_t b, uint64_t e) {
  while (e > b && fq_space((unsigned char)s[e - 1])) e--;
  return e;
}

// get_fq_name's verdict (src/fastq.cpp:73-122) on the trimmed id line [b, e), which starts with '@'.
// The header is scanned 16 bytes at a time (16 independent loads, then the tests) so that a lane waits for
// one memory round trip per 16 characters instead of one per character.
__device__ bool name_ok(const char *s, uint64_t b, uint64_t e) {
  const char *h = s + b + 1;
  const uint64_t len = rtrim_end(s, b + 1, e) - (b + 1);
  if (len < 3 || h[len - 2] == '/') return true;
  if (h[len - 2] == 'R') return true;  // HudsonAlpha @pair-R1 / @pair-R2
  uint64_t tab = len, sp = len;
  for (uint64_t i0 = 0; i0 < len && tab == len; i0 += 16) {
    char v[16];
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = i0 + j < len ? h[i0 + j] : 'x';
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (v[j] == '\t' && tab == len) tab = i0 + j;
      if (v[j] == ' ' && sp == len) sp = i0 + j;
    }
  }
  const uint64_t ep = tab < len ? tab : sp;  // first tab, else first space
  if (ep == len) return true;                // no comment
  if (ep > 3 && h[ep - 2] == '/' && (h[ep - 1] == '1' || h[ep - 1] == '2')) return true;
  if (len < ep + 7 || h[ep + 2] != ':' || h[ep + 4] != ':' || h[ep + 6] != ':' || (h[ep + 1] != '1' && h[ep + 1] != '2'))
    return false;
  return true;
}

__device__ __forceinline__ void fq_fail(unsigned long long *err, uint64_t r, int kind) {
  atomicMin(err, ((unsigned long long)r << 4) | (unsigned long long)kind);
}

__global__ __launch_bounds__(FQ_THREADS) void k_fq_records(const char *text, uint64_t n,
                                                            const unsigned long long *line_end, uint64_t n_rec,
                                                            unsigned long long *len, unsigned long long *err) {
  const uint64_t r = (uint64_t)blockIdx.x * FQ_THREADS + threadIdx.x;
  if (r > n_rec) return;
  if (r == n_rec) {  // the scan's last element: offs[n_rec] = total
    len[r] = 0;
    return;
  }
  uint64_t lw[5], lb[4], le[4], te[4];
#pragma unroll
  for (int i = 0; i < 5; i++) lw[i] = (4 * r + i) ? line_end[4 * r + i - 1] : 0;  // lw[i]: the word ending line 4r+i-1
#pragma unroll
  for (int i = 0; i < 4; i++) {
    lb[i] = (4 * r + i) ? (lw[i] & FQ_LE_MASK) + 1 : 0;
    le[i] = lw[i + 1] & FQ_LE_MASK;
    // a last line without a newline (end = n, set by the host) has no metadata of its own
    te[i] = le[i] == n ? rtrim_end(text, lb[i], le[i]) : le[i] - ((lw[i + 1] >> FQ_LE_BITS) & 0xffffu);
  }
  len[r] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (le[i] - lb[i] > FQ_MAX_LINE) return fq_fail(err, r, FQ_E_LONG);
  // first characters of the id and '+' lines (the following newline when a line is empty)
  const unsigned char c_id = r ? (unsigned char)(lw[0] >> 56) : (n ? (unsigned char)text[0] : 0);
  const unsigned char c_plus = (unsigned char)(lw[2] >> 56);
  if (te[0] == lb[0] || c_id != '@') return fq_fail(err, r, FQ_E_ID);
  if (le[2] == lb[2] || c_plus != '+') return fq_fail(err, r, FQ_E_PLUS);
  if (!name_ok(text, lb[0], te[0])) return fq_fail(err, r, FQ_E_NAME);
  const uint64_t L = te[1] - lb[1];
  if (L != te[3] - lb[3]) return fq_fail(err, r, FQ_E_LEN);
  len[r] = L;
}

// PackedRead base code (packed_reads.cpp:87-105), -1 for a fatal character
__device__ __forceinline__ int base_code(unsigned char c) {
  const uint32_t i = (uint32_t)c - 'A';
  if (i >= 26) return -1;
  if (i == 0) return 0;
  if (i == 'C' - 'A') return 1;
  if (i == 'G' - 'A') return 2;
  if (i == 'T' - 'A') return 3;
  constexpr uint32_t four = (1u << ('N' - 'A')) | (1u << ('U' - 'A')) | (1u << ('R' - 'A')) | (1u << ('Y' - 'A')) |
                            (1u << ('K' - 'A')) | (1u << ('M' - 'A')) | (1u << ('S' - 'A')) | (1u << ('W' - 'A')) |
                            (1u << ('B' - 'A')) | (1u << ('D' - 'A')) | (1u << ('H' - 'A')) | (1u << ('V' - 'A'));
  return ((four >> i) & 1u) ? 4 : -1;
}

// One 16-lane group per record. The group walks the record in runs of 64 bases: lane t owns output
// dword d = 16 * run + t. It reads bases [4d, 4d + 4) of the sequence and quality lines as two aligned
// dwords joined with v_alignbyte (the text lines start at any byte), packs them into W_d, and writes the
// ALIGNED output dword that holds record bytes [4d - s, 4d + 4 - s), s = the record's output misalignment:
// the high s bytes of W_{d-1} (the next lower lane, row_shr:1 DPP; lane 0 takes the previous run's lane 15)
// and the low 4 - s bytes of W_d. Only the record's first and last dwords, which it shares with its
// neighbours, are written bytewise. (Unaligned dwordx4 loads and stores, which gfx950's unaligned-access
// mode allows, measured slower: 4.6 ms vs 3.2 ms for byte stores at C2.) A dword that starts inside the
// text is read whole: allocations are at least 4-byte granular.
constexpr int FQ_GROUP = 16;
__device__ __forceinline__ uint32_t load4(const char *text, uint32_t a) {
  const uintptr_t p = (uintptr_t)(text + a);  // aligned in the address space, not relative to text
  const uint32_t *w = (const uint32_t *)(p & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(p & 3u);
  const uint32_t v0 = w[0];
  if (sh == 0) return v0;
  return __builtin_amdgcn_alignbyte(w[1], v0, sh);  // v_alignbyte_b32: ({w1, v0} >> 8 * sh)
}
// exact per-byte zero test: bit 7 of each byte of the result is set iff that byte of x is 0
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t pack4(uint32_t vs, uint32_t vq, int n_valid, int qual_offset, bool &bad) {
  // SWAR fast path: four A/C/G/T bases with qualities in [qual_offset, 0x7f]
  const uint32_t acgt = zero_bytes(vs ^ 0x41414141u) | zero_bytes(vs ^ 0x43434343u) | zero_bytes(vs ^ 0x47474747u) |
                        zero_bytes(vs ^ 0x54545454u);
  const uint32_t qo = (uint32_t)qual_offset * 0x01010101u;
  const bool q_ok = (vq & 0x80808080u) == 0 && (((vq | 0x80808080u) - qo) & 0x80808080u) == 0x80808080u;
  if (n_valid >= 4 && acgt == 0x80808080u && q_ok) {
    uint32_t code = (vs >> 1) & 0x03030303u;  // A 0, C 1, G 3, T 2
    code ^= (code >> 1) & 0x01010101u;        // G 2, T 3
    uint32_t x = vq - qo;                     // q - offset per byte, no borrows
    uint32_t over = x & 0x60606060u;          // q - offset >= 32 (< 0x80): bit 5 or 6
    over = ((over | (over >> 1)) >> 5) & 0x01010101u;
    x = (x & ~(over * 0xffu)) | (over * 31u);  // min(q - offset, 31)
    return code | (x << 3);
  }
  uint32_t w = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const bool in = j < n_valid;
    const int c = base_code(in ? (unsigned char)(vs >> (8 * j)) : 'A');
    int q = (int)(signed char)(vq >> (8 * j)) - qual_offset;
    q = q < 31 ? q : 31;
    bad |= c < 0;
    const uint32_t byte = (uint32_t)(uint8_t)((c & 7) | (uint8_t)((unsigned)(unsigned char)q << 3));
    w |= in ? byte << (8 * j) : 0u;
  }
  return w;
}
__global__ __launch_bounds__(FQ_THREADS) void k_fq_pack(const char *text, const unsigned long long *line_end,
                                                         uint64_t n_rec, const unsigned long long *offs,
                                                         int qual_offset, uint8_t *out, unsigned long long *err) {
  const uint64_t r = (uint64_t)blockIdx.x * (FQ_THREADS / FQ_GROUP) + (threadIdx.x / FQ_GROUP);
  const int gl = threadIdx.x % FQ_GROUP;
  const int last_of_group = (threadIdx.x & 63 & ~(FQ_GROUP - 1)) + FQ_GROUP - 1;
  bool bad = false;
  // every lane of the wave takes part in the cross-lane moves: no early exit
  const bool live = r < n_rec;
  const char *sp = text, *qp = text;
  uint8_t *dst = out;
  int L = 0;
  if (live) {
    // 32-bit offsets inside a record (lines are at most FQ_MAX_LINE long): one 64-bit base per stream
    sp = text + (line_end[4 * r] & FQ_LE_MASK) + 1;
    qp = text + (line_end[4 * r + 2] & FQ_LE_MASK) + 1;
    const uint64_t o = offs[r];
    dst = out + o;
    L = (int)(offs[r + 1] - o);
  }
  const int s = (int)((uintptr_t)dst & 3u);
  uint32_t *const a0 = (uint32_t *)((uintptr_t)dst - (uintptr_t)s);  // aligned; dword d covers [4d - s, 4d + 4 - s)
  // the group's runs: while the run's first aligned dword starts inside the record (uniform per wave: the
  // longest record of the wave's groups decides, idle groups run with L = 0)
  int wave_L = L;
#pragma unroll
  for (int d = 16; d < 64; d <<= 1) wave_L = max(wave_L, __shfl_xor(wave_L, d, 64));
  uint32_t carry = 0;  // W_{-1} of the next run's lane 0
  // (hoisting the loads of 4 runs ahead of their use measured slower: 3.38 vs 3.09 ms at C2)
  for (int base = 0; 4 * base - 3 < wave_L; base += FQ_GROUP) {
    const int d = base + gl, i = 4 * d;
    uint32_t vs = 0x41414141u, vq = 0;
    if (i < L) {
      vs = load4(sp, (uint32_t)i);
      vq = load4(qp, (uint32_t)i);
    }
    const uint32_t w = pack4(vs, vq, min(4, L - i), qual_offset, bad);
    // W_{d-1}: row_shr:1 within the 16-lane row; lane 0 of the row keeps 'old' = carry
    const uint32_t wm = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)w, 0x111, 0xf, 0xf, false);
    carry = (uint32_t)__shfl((int)w, last_of_group, 64);
    const uint32_t ow = s ? __builtin_amdgcn_alignbyte(w, wm, 4 - s) : w;
    const int x0 = i - s;  // record byte of the output dword's first byte
    if (x0 >= 0 && x0 + 4 <= L) {
      a0[d] = ow;
    } else if (x0 < L && x0 + 4 > 0) {  // the record's first or last dword: only its own bytes
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (x0 + j >= 0 && x0 + j < L) ((uint8_t *)(a0 + d))[j] = (uint8_t)(ow >> (8 * j));
    }
  }
  // groups of a wave hold consecutive records: the lowest bad record of the wave is reported (atomicMin)
  const uint64_t bal = __ballot(bad);
  if (bal && (threadIdx.x & 63) == 0) {
    const int first_lane = __ffsll((long long)bal) - 1;
    fq_fail(err, (uint64_t)blockIdx.x * (FQ_THREADS / FQ_GROUP) + ((threadIdx.x & ~63) + first_lane) / FQ_GROUP,
            FQ_E_CHAR);
  }
}

}  // namespace

size_t fq_scan_tmp_bytes(uint64_t n_items) {
  size_t a = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const unsigned long long *)nullptr, (unsigned long long *)nullptr, 0ull,
                                (size_t)n_items, rocprim::plus<unsigned long long>());
  return a;
}

hipError_t fq_scan(void *tmp, size_t tmp_bytes, const unsigned long long *in, unsigned long long *out,
                   uint64_t n_items, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, 0ull, (size_t)n_items, rocprim::plus<unsigned long long>(), s);
}

hipError_t launch_fq_count(const char *text, uint64_t n, unsigned long long *chunk, hipStream_t s) {
  const uint64_t nch = (n + FQ_CHUNK - 1) / FQ_CHUNK;
  if (nch) hipLaunchKernelGGL(k_fq_count, dim3((uint32_t)nch), dim3(FQ_THREADS), 0, s, text, n, chunk);
  return hipGetLastError();
}

hipError_t launch_fq_lines(const char *text, uint64_t n, const unsigned long long *chunk_base,
                           unsigned long long *line_end, hipStream_t s) {
  const uint64_t nch = (n + FQ_CHUNK - 1) / FQ_CHUNK;
  if (nch) hipLaunchKernelGGL(k_fq_lines, dim3((uint32_t)nch), dim3(FQ_THREADS), 0, s, text, n, chunk_base, line_end);
  return hipGetLastError();
}

hipError_t launch_fq_records(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_rec,
                             unsigned long long *len, unsigned long long *err, hipStream_t s) {
  const uint64_t nb = (n_rec + 1 + FQ_THREADS - 1) / FQ_THREADS;
  hipLaunchKernelGGL(k_fq_records, dim3((uint32_t)nb), dim3(FQ_THREADS), 0, s, text, n, line_end, n_rec, len, err);
  return hipGetLastError();
}

hipError_t launch_fq_pack(const char *text, const unsigned long long *line_end, uint64_t n_rec,
                          const unsigned long long *offs, int qual_offset, uint8_t *out, unsigned long long *err,
                          hipStream_t s) {
  const uint64_t nb = (n_rec + FQ_THREADS / FQ_GROUP - 1) / (FQ_THREADS / FQ_GROUP);
  if (nb)
    hipLaunchKernelGGL(k_fq_pack, dim3((uint32_t)nb), dim3(FQ_THREADS), 0, s, text, line_end, n_rec, offs,
                       qual_offset, out, err);
  return hipGetLastError();
}

}  // namespace mhm
