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

#include <algorithm>

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

// Inclusive prefix sum over the wave: DPP row shifts within the 16-lane rows, then the GFX9 row broadcasts
// (row_bcast:15, row_bcast:31) across them; six VALU moves instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
  const int rl = lane & 15;
  uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (rl >= 1) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (rl >= 2) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (rl >= 4) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  if (rl >= 8) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x142, 0xf, 0xf, false);  // row_bcast:15
  if (lane & 16) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x143, 0xf, 0xf, false);  // row_bcast:31
  if (lane >= 32) v += t;
  return v;
}

__global__ __launch_bounds__(FQ_THREADS) void k_fq_count(const char *text, uint64_t n, unsigned long long *chunk) {
  __shared__ uint32_t s_w[FQ_THREADS / 64];
  const uint64_t pos = (uint64_t)blockIdx.x * FQ_CHUNK + (uint64_t)threadIdx.x * FQ_BYTES;
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(__popc(nl_mask(text, pos, n)), threadIdx.x & 63), 63);
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
  const uint32_t incl = wave_incl_scan(c, lane);
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint64_t o = chunk_base[blockIdx.x] + (incl - c);
  for (int w = 0; w < wid; w++) o += s_w[w];
  // the neighbouring lanes' edge bytes (the byte before this lane's 16 and the byte after them), so that
  // only the wave's edge lanes go to memory for them
  const uint32_t prev_w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[3], 0x138, 0xf, 0xf, false);  // wave_shr:1
  const uint32_t next_w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[0], 0x130, 0xf, 0xf, false);  // wave_shl:1
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
  // aligned in the address space, not relative to text; the dword pointer is derived from text (not rebuilt
  // from an integer) so that the compiler keeps global loads instead of flat ones
  const char *p = text + a;
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
  const uint32_t *w = (const uint32_t *)(p - sh);
  // the second dword only when the four bytes straddle one, without a branch (the address is selected)
  return __builtin_amdgcn_alignbyte(*(sh ? w + 1 : w), w[0], sh);  // v_alignbyte_b32: ({w1, w0} >> 8 * sh)
}
// exact per-byte zero test: bit 7 of each byte of the result is set iff that byte of x is 0
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
// Byte classification by v_perm_b32 lookups: the low three bits of A C T N G (1 3 4 6 7) are distinct, so
// one 8-entry byte table indexed by them gives a candidate answer and a second gives the character that index
// stands for; a byte is A/C/G/T/N exactly when it equals that character. No per-byte branches: the switch-like
// compare chains these replace compiled to divergent branch trees, and k_fq_merge was bound by SALU issue.
__device__ __forceinline__ uint32_t perm8(uint64_t table, uint32_t sel) {
  return __builtin_amdgcn_perm((uint32_t)(table >> 32), (uint32_t)table, sel);
}
constexpr uint64_t byte_table(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, uint32_t v4, uint32_t v5, uint32_t v6,
                              uint32_t v7) {
  return (uint64_t)v0 | (uint64_t)v1 << 8 | (uint64_t)v2 << 16 | (uint64_t)v3 << 24 | (uint64_t)v4 << 32 |
         (uint64_t)v5 << 40 | (uint64_t)v6 << 48 | (uint64_t)v7 << 56;
}
// index (low 3 bits):          0     1    2     3    4    5     6    7
constexpr uint64_t T_CHAR = byte_table(0x01, 'A', 0x01, 'C', 'T', 0x01, 'N', 'G');  // 0x01: matches no byte there
constexpr uint64_t T_CODE5 = byte_table(0, 0, 0, 1, 3, 0, 4, 2);  // PackedRead base codes: A 0, C 1, G 2, T 3, N 4
constexpr uint64_t T_CODE2 = byte_table(0, 0, 0, 1, 3, 0, 0, 2);
constexpr uint64_t T_FLAG = byte_table(0, 0, 0, 0, 0, 0, 1, 0);
constexpr uint64_t T_COMP = byte_table(0, 'T', 0, 'G', 'A', 0, 'N', 'C');
// 0x01 in every byte of w that is one of A C G T N, 0 elsewhere
__device__ __forceinline__ uint32_t acgtn_bytes(uint32_t w, uint32_t sel) {
  return zero_bytes(w ^ perm8(T_CHAR, sel)) >> 7;
}
// bit 7 of every byte of w equal to v (v replicated), 0 elsewhere
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t v4) { return zero_bytes(w ^ v4); }
__device__ __forceinline__ uint32_t pack4(uint32_t vs, uint32_t vq, int n_valid, int qual_offset, bool &bad) {
  // SWAR fast path: A/C/G/T/N bases (codes by table, as nib and comp) with qualities in [qual_offset, 0x7f]; bytes
  // past n_valid count as 'A' with quality qual_offset and come out 0, so a record's last word takes it too
  const uint32_t qo = (uint32_t)qual_offset * 0x01010101u;
  const uint32_t vm = n_valid >= 4 ? ~0u : (1u << (8 * n_valid)) - 1u;  // the valid bytes (n_valid >= 1)
  const uint32_t s = (vs & vm) | (0x41414141u & ~vm), q = (vq & vm) | (qo & ~vm);
  const uint32_t sel = s & 0x07070707u;
  const bool q_ok = (q & 0x80808080u) == 0 && (((q | 0x80808080u) - qo) & 0x80808080u) == 0x80808080u;
  if (acgtn_bytes(s, sel) == 0x01010101u && q_ok) {
    const uint32_t code = perm8(T_CODE5, sel);  // A 0, C 1, G 2, T 3, N 4
    uint32_t x = q - qo;                        // q - offset per byte, no borrows
    uint32_t over = x & 0x60606060u;            // q - offset >= 32 (< 0x80): bit 5 or 6
    over = ((over | (over >> 1)) >> 5) & 0x01010101u;
    x = (x & ~(over * 0xffu)) | (over * 31u);  // min(q - offset, 31)
    return (code | (x << 3)) & vm;
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
    // every lane loads (clamped into the record; an idle group's L = 0 reads the text's first dword) and packs;
    // lanes past the record keep 0 and raise no error
    const int ic = min(i, max(L - 1, 0));
    const uint32_t vs = load4(sp, (uint32_t)ic), vq = load4(qp, (uint32_t)ic);
    bool bw = false;
    const uint32_t pw = pack4(vs, vq, max(1, min(4, L - i)), qual_offset, bw);
    const uint32_t w = i < L ? pw : 0u;
    bad |= bw && i < L;
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

// ------------------------------------------------------------------------------------------------
// Read-pair merging (merge_reads, src/merge_reads.cpp:237-588) of an interleaved paired FASTQ text: records 2p
// and 2p+1 are the mates of pair p (FastqReader interleaves a pair of files the same way, fastq.cpp:509-516).
// k_fq_merge (one lane per pair) checks the pair's names, scans the offsets of the reverse-complemented mate 2
// against mate 1 exactly as the reference does and records the verdict; k_fq_merge_pack (one 16-lane group
// per output read) writes merge_reads' PackedReads: the merged read and a dummy "N" mate, or both mates.
// The scan only ever changes qualities at N bases (an N's quality becomes the offset, :371-383), which the
// output keeps; pairs with an N therefore scan copies of their quality lines in a scratch laid out like the
// packed records (mate 1's qualities, mate 2's reversed), the others read the text in place.

// Q2Perror (merge_reads.cpp:73-81), 81 entries
__constant__ double Q2P_TAB[81] = {
    1.0,       0.7943,    0.6309,    0.5012,    0.3981,    0.3162,    0.2512,    0.1995,    0.1585,    0.1259,     0.1,
    0.07943,   0.06310,   0.05012,   0.03981,   0.03162,   0.02512,   0.01995,   0.01585,   0.01259,   0.01,       0.007943,
    0.006310,  0.005012,  0.003981,  0.003162,  0.002512,  0.001995,  0.001585,  0.001259,  0.001,     0.0007943,  0.0006310,
    0.0005012, 0.0003981, 0.0003162, 0.0002512, 0.0001995, 0.0001585, 0.0001259, 0.0001,    7.943e-05, 6.310e-05,  5.012e-05,
    3.981e-05, 3.162e-05, 2.512e-05, 1.995e-05, 1.585e-05, 1.259e-05, 1e-05,     7.943e-06, 6.310e-06, 5.012e-06,  3.981e-06,
    3.162e-06, 2.512e-06, 1.995e-06, 1.585e-06, 1.259e-06, 1e-06,     7.943e-07, 6.310e-07, 5.012e-07, 3.981e-07,  3.1622e-07,
    2.512e-07, 1.995e-07, 1.585e-07, 1.259e-07, 1e-07,     7.943e-08, 6.310e-08, 5.012e-08, 3.981e-08, 3.1622e-08, 2.512e-08,
    1.995e-08, 1.585e-08, 1.259e-08, 1e-08};

// A record's lines: id [idb, idte), sequence [sb, sb + L), quality [qb, qb + L) (fq_record_check)
struct FqRec {
  uint64_t idb, idte, sb, qb;
  uint32_t L;
};

// get_fq_name + replace_spaces (fastq.cpp:73-122, :544): the normalized name of the trimmed id line [b, e) as
// prefix [pb, pe) (the name without its last two characters) and the last character
__device__ bool fq_norm(const char *s, uint64_t b, uint64_t e, uint64_t &pb, uint64_t &pe, char &last) {
  const char *h = s + b + 1;
  const uint64_t len = rtrim_end(s, b + 1, e) - (b + 1);
  pb = b + 1;
  if (len >= 3 && h[len - 2] != '/') {
    if (h[len - 2] == 'R') {  // pair-R1 -> pair/1
      pe = b + 1 + len - 3;
      last = h[len - 1];
      return true;
    }
    uint64_t tab = len, sp = len;
    for (uint64_t i0 = 0; i0 < len && tab == len; i0 += 16) {  // 16 independent loads per step, as name_ok
      char v[16];
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = i0 + j < len ? h[i0 + j] : 'x';
#pragma unroll
      for (int j = 0; j < 16; j++) {
        if (v[j] == '\t' && tab == len) tab = i0 + j;
        if (v[j] == ' ' && sp == len) sp = i0 + j;
      }
    }
    const uint64_t ep = tab < len ? tab : sp;
    if (ep == len) {  // no comment: unchanged
      pe = b + 1 + len - 2;
      last = h[len - 1];
      return true;
    }
    if (ep > 3 && h[ep - 2] == '/' && (h[ep - 1] == '1' || h[ep - 1] == '2')) {
      pe = b + 1 + ep - 2;
      last = h[ep - 1];
      return true;
    }
    if (len < ep + 7 || h[ep + 2] != ':' || h[ep + 4] != ':' || h[ep + 6] != ':' || (h[ep + 1] != '1' && h[ep + 1] != '2'))
      return false;
    pe = b + 1 + ep;  // pair 1:N:... -> pair/1
    last = h[ep + 1];
    return true;
  }
  pe = b + 1 + (len >= 2 ? len - 2 : 0);
  last = len ? h[len - 1] : 0;
  return true;
}

// per pair: (overlap + 1) of the merge (0: not merged) | has-N << 31
constexpr uint32_t MP_HASN = 1u << 31;

// Where a pair's lines are (k_fq_pair_records); L1 = ~0: the pair is not merged (a record or name error, which
// is reported)
struct PairDesc {
  uint64_t s1, q1, s2, q2;
  uint32_t L1, L2;
};

// Pairs whose mates are both at most MG_LONG bases (every short-read run) go through a k_fq_merge instance with
// MG_SHORT-byte staging: 11 KB of LDS per workgroup instead of 42 KB, so MG_OCC workgroups per CU instead of
// three hide each other's LDS and shuffle round trips. k_fq_pair_records lists the other pairs (after the
// descriptors: a counter, then the pair indices), which a launch of the 2048-byte instance takes.
constexpr int MG_SHORT = 512;
constexpr int MG_OCC = 8;
constexpr uint32_t MG_LONG = (uint32_t)MG_SHORT - 8;  // longest mate of a short pair
__host__ __device__ inline uint32_t *long_pairs(void *desc_buf, uint64_t n_pairs) {  // [counter, 15 pad, list]
  return (uint32_t *)((char *)desc_buf + (((size_t)n_pairs * sizeof(PairDesc) + 63) & ~(size_t)63));
}

// Paired input: the records' checks (as k_fq_records) and the pairs' descriptors in one pass, one lane per pair
// (until round 4 a separate k_fq_pair_prep re-read every id line and line-end word). Each record gets
// k_fq_records' checks, length and errors (the id line's get_fq_name verdict is fq_norm's, which also gives the
// name to compare); then the pair's names (replace_spaces: spaces read as '_', four characters per load) and
// pair numbers are checked (:320-321) and its descriptor written. A trailing unpaired record (odd count) is
// checked as a record only.
__device__ bool fq_record_check(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t r,
                                unsigned long long *len, unsigned long long *err, FqRec &o, uint64_t &pb, uint64_t &pe,
                                char &last) {
  uint64_t lw[5], lb[4], le[4], te[4];
#pragma unroll
  for (int i = 0; i < 5; i++) lw[i] = (4 * r + i) ? line_end[4 * r + i - 1] : 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    lb[i] = (4 * r + i) ? (lw[i] & FQ_LE_MASK) + 1 : 0;
    le[i] = lw[i + 1] & FQ_LE_MASK;
    te[i] = le[i] == n ? rtrim_end(text, lb[i], le[i]) : le[i] - ((lw[i + 1] >> FQ_LE_BITS) & 0xffffu);
  }
  len[r] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (le[i] - lb[i] > FQ_MAX_LINE) {
      fq_fail(err, r, FQ_E_LONG);
      return false;
    }
  const unsigned char c_id = r ? (unsigned char)(lw[0] >> 56) : (n ? (unsigned char)text[0] : 0);
  const unsigned char c_plus = (unsigned char)(lw[2] >> 56);
  if (te[0] == lb[0] || c_id != '@') {
    fq_fail(err, r, FQ_E_ID);
    return false;
  }
  if (le[2] == lb[2] || c_plus != '+') {
    fq_fail(err, r, FQ_E_PLUS);
    return false;
  }
  if (!fq_norm(text, lb[0], te[0], pb, pe, last)) {
    fq_fail(err, r, FQ_E_NAME);
    return false;
  }
  const uint64_t L = te[1] - lb[1];
  if (L != te[3] - lb[3]) {
    fq_fail(err, r, FQ_E_LEN);
    return false;
  }
  len[r] = L;
  o.idb = lb[0];
  o.idte = te[0];
  o.sb = lb[1];
  o.qb = lb[3];
  o.L = (uint32_t)L;
  return true;
}
__global__ __launch_bounds__(FQ_THREADS) void k_fq_pair_records(const char *text, uint64_t n,
                                                                 const unsigned long long *line_end, uint64_t n_rec,
                                                                 unsigned long long *len, unsigned long long *err,
                                                                 PairDesc *desc, uint32_t *long_list) {
  const uint64_t p = (uint64_t)blockIdx.x * FQ_THREADS + threadIdx.x, r0 = 2 * p;
  if (r0 > n_rec) return;
  if (r0 == n_rec) {  // the scan's last element: offs[n_rec] = total
    len[n_rec] = 0;
    return;
  }
  FqRec a, b;
  uint64_t pb1 = 0, pe1 = 0, pb2 = 0, pe2 = 0;
  char l1 = 0, l2 = 0;
  const bool ok1 = fq_record_check(text, n, line_end, r0, len, err, a, pb1, pe1, l1);
  if (r0 + 1 == n_rec) {  // an unpaired last record; the scan's last element
    len[n_rec] = 0;
    return;
  }
  const bool ok2 = fq_record_check(text, n, line_end, r0 + 1, len, err, b, pb2, pe2, l2);
  PairDesc d{0, 0, 0, 0, ~0u, 0};
  if (ok1 && ok2) {
    bool same = pe1 - pb1 == pe2 - pb2;
    for (uint64_t i = 0; same && i < pe1 - pb1; i += 4) {
      const uint64_t left = pe1 - pb1 - i;
      const uint32_t valid = left >= 4 ? ~0u : (1u << (8 * left)) - 1;
      uint32_t x = load4(text + pb1, (uint32_t)i), y = load4(text + pb2, (uint32_t)i);
      const uint32_t sx = (zero_bytes(x ^ 0x20202020u) >> 7) * 0xffu, sy = (zero_bytes(y ^ 0x20202020u) >> 7) * 0xffu;
      x = (x & ~sx) | (0x5f5f5f5fu & sx);
      y = (y & ~sy) | (0x5f5f5f5fu & sy);
      same = ((x ^ y) & valid) == 0;
    }
    if (!same) {
      fq_fail(err, 2 * p + 1, FQ_E_PAIR_NAME);
    } else if (l1 != '1' || l2 != '2') {
      fq_fail(err, 2 * p + 1, FQ_E_PAIR_NUM);
    } else {
      d = PairDesc{a.sb, a.qb, b.sb, b.qb, a.L, b.L};
      if (a.L > MG_LONG || b.L > MG_LONG) long_list[16 + atomicAdd(long_list, 1u)] = (uint32_t)p;
    }
  }
  desc[p] = d;
}

// One wave per pair (grid-stride). The pair is staged in the wave's LDS: mate 1's bases and qualities, mate
// 2 reverse-complemented (RC) with its reversed qualities (RQ). Then
//   1. fast filter (fast_count_mismatches, :183-230): lane t takes the offsets t, t + 64, ..., comparing four
//      bytes at a time with an early exit; a ballot keeps the offsets with at most error_max_mismatch;
//   2. the kept offsets, in increasing order, get the reference's base-by-base scan (:357-427), evaluated across
//      the lanes: per position its match / mismatch / N increments, wave prefix sums of them find the position
//      where the reference breaks (a second both-N, more than 3 N, too many mismatches, a bad quality), and the
//      error-probability sum is added up position by position in the reference's order (double, two adds per
//      N mismatch as there);
//   3. the good / weak / ambiguous bookkeeping of :428-444 runs over those verdicts in order.
// A scan's effect on qualities (an N's quality becomes the offset) does not change any later verdict: the
// quality read at an N is always the one just set. It does change the output, so it is applied in LDS in scan
// order and the qualities of pairs with an N go to the scratch for k_fq_merge_pack.
constexpr int MG_WAVES = 4;
constexpr int MG_MAXL = 2048;  // > FQ_MAX_LINE + 4 (unaligned 4-byte reads past a line stay inside)

// The fast filter's view of four characters: 2-bit codes (A C G T = 0..3, N and the rest 0) and 2-bit flags
// (N 1, a character other than A C G T N 2, else 0), one byte each, first character in the low bits. Two
// characters are equal exactly when both their codes and their flags are.
__device__ __forceinline__ uint32_t pack2x4(uint32_t v) {  // four 2-bit values, one per byte, into one byte
  const uint32_t t = v | (v >> 6);
  return (t & 0xfu) | ((t >> 12) & 0xf0u);
}
__device__ __forceinline__ void codes_flags4(uint32_t w, uint32_t &code, uint32_t &flag) {
  const uint32_t sel = w & 0x07070707u, ok = acgtn_bytes(w, sel);
  code = pack2x4(perm8(T_CODE2, sel) & (ok * 0xffu));
  flag = pack2x4((perm8(T_FLAG, sel) & (ok * 0xffu)) | ((ok ^ 0x01010101u) * 2u));
}
// fq_comp of every byte of w (A<->T, C<->G, N and IUPAC -> N, anything else 0)
__device__ __forceinline__ uint32_t comp4(uint32_t w) {
  const uint32_t sel = w & 0x07070707u, ok = acgtn_bytes(w, sel);
  uint32_t out = perm8(T_COMP, sel) & (ok * 0xffu);
  if (ok != 0x01010101u) {  // another character: IUPAC codes complement to N (utils.cpp revcomp), the rest to 0
    constexpr uint32_t NI = (1u << ('N' - 'A')) | (1u << ('U' - 'A')) | (1u << ('R' - 'A')) | (1u << ('Y' - 'A')) |
                            (1u << ('K' - 'A')) | (1u << ('M' - 'A')) | (1u << ('S' - 'A')) | (1u << ('W' - 'A')) |
                            (1u << ('B' - 'A')) | (1u << ('D' - 'A')) | (1u << ('H' - 'A')) | (1u << ('V' - 'A'));
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t k = ((w >> (8 * i)) & 0xffu) - 'A';
      if (!((ok >> (8 * i)) & 1u) && k < 26u && ((NI >> k) & 1u)) out |= (uint32_t)'N' << (8 * i);
    }
  }
  return out;
}
__device__ __forceinline__ int nz_bytes(uint32_t x) {  // bytes of x that are not zero
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return __popc(x & 0x01010101u);
}
// the lanes below this one whose bit is set in m (v_mbcnt_lo / v_mbcnt_hi)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// lane l's value (l uniform): v_readlane into a scalar register, no LDS round trip as __shfl's ds_bpermute
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double lane_f64(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned long long lo = lane_u32((uint32_t)b, l), hi = lane_u32((uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)((hi << 32) | lo));
}
// The lane index, recomputed where it is called: the compiler cannot hoist the lane-derived LDS addresses of a
// loop body built from it out of the loop (in k_fq_merge's pair loop they took a dozen VGPRs for the whole
// kernel and pushed it into spills at 80 VGPRs).
__device__ __forceinline__ int opaque_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MAXL < MG_MAXL: the pairs with a mate longer than MG_LONG are left to the MG_MAXL instance, which (given
// long_list) takes only the listed pairs.
template <int MAXL>
__global__ __launch_bounds__(64 * MG_WAVES, MAXL < MG_MAXL ? MG_OCC : 3) void k_fq_merge(
    const char *text, const PairDesc *desc, uint64_t n_pairs, const unsigned long long *rec_offs, int qual_offset,
    char *scratch, uint32_t *pair_info, unsigned long long *out_len, unsigned long long *err,
    unsigned long long *stats, const uint32_t *long_list) {
  __shared__ __align__(16) char lds[MG_WAVES][4][MAXL + 16];
  // the bases again as 2-bit codes and 2-bit flags (codes_flags4), 32 per word, for the fast filter's 32-base
  // compares: [wave][S1 codes, S1 flags, RC codes, RC flags][word]
  __shared__ __align__(16) uint64_t cf[MG_WAVES][4][MAXL / 32 + 4];
  // Q2Perror in LDS: a mismatch's table reads are divergent, and from constant memory each was a memory round
  // trip on the scan's critical path
  __shared__ double q2p[81];
  for (int t = threadIdx.x; t < 81; t += blockDim.x) q2p[t] = Q2P_TAB[t];
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // (w scalar: scalar pair loads)
  char *S1 = lds[w][0], *RC = lds[w][1], *Q1 = lds[w][2], *RQ = lds[w][3];
  uint64_t *S1c = cf[w][0], *S1f = cf[w][1], *RCc = cf[w][2], *RCf = cf[w][3];
  const int16_t MIN_OVERLAP = 12, EXTRA_TEST_OVERLAP = 2, MAX_MISMATCHES = 3, EXTRA_PER_1000 = 150;
  const double MAX_PERROR = 0.025;
  uint64_t merged = 0, ambiguous = 0, ov_bases = 0;
  const uint64_t n_waves = (uint64_t)gridDim.x * MG_WAVES;
  if (blockIdx.x == 0 && threadIdx.x == 0) out_len[2 * n_pairs] = 0;  // the scan's last element
  const uint64_t n_items = long_list ? long_list[0] : n_pairs;
  // The next pair's index and descriptor are loaded (scalar loads) while this pair is worked: a pair starts with
  // its text loads, not with a descriptor round trip before them.
  const uint64_t it0 = (uint64_t)blockIdx.x * MG_WAVES + w;
  uint64_t pn = 0;
  PairDesc dn{0, 0, 0, 0, ~0u, 0};
  if (it0 < n_items) {
    pn = long_list ? long_list[16 + it0] : it0;
    dn = desc[pn];
  }
  for (uint64_t it = it0; it < n_items; it += n_waves) {
    const int lane = opaque_lane();
    const uint64_t p = pn;
    const PairDesc d = dn;
    if (it + n_waves < n_items) {
      pn = long_list ? long_list[16 + it + n_waves] : it + n_waves;
      dn = desc[pn];
    }
    const bool is_long = d.L1 != ~0u && (d.L1 > MG_LONG || d.L2 > MG_LONG);
    if (MAXL < MG_MAXL && is_long) continue;  // (listed for the MG_MAXL instance, which initialises its outputs)
    if (lane == 0) {
      pair_info[p] = 0;
      out_len[2 * p] = 0;
      out_len[2 * p + 1] = 0;
    }
    if (d.L1 == ~0u) continue;  // (its error is reported)
    const int L1 = (int)d.L1, L2 = (int)d.L2;
    const char *s1 = text + d.s1, *tq1 = text + d.q1, *s2 = text + d.s2, *tq2 = text + d.q2;
    // staging, four bytes per lane and step (one load round trip for reads up to 256 bases); a step may read
    // up to three bytes before or after a line, which are text (the id line before it, the newline after it)
    bool bad2 = false, hasN = false;
    // both mates in one uniform loop: every lane loads (addresses clamped into the lines) and classifies, only the
    // stores are masked (per-lane trip counts had the loops' exec masks saved and restored every step)
    const int LM = L1 > L2 ? L1 : L2;
    for (int b = 0; b < LM; b += 256) {
      const int x0 = b + 4 * lane;
      const int xs = min(x0, L1 - 1), js = min(x0, L2 - 1);
      const uint32_t c = load4(s1, (uint32_t)xs), q = load4(tq1, (uint32_t)xs);
      const int a0 = L2 - 4 - js;  // s2 bytes a0 .. a0 + 3 are RC[js + 3] .. RC[js]
      const uint32_t rc = comp4(__builtin_bswap32(load4(s2 + a0, 0u))), rq = __builtin_bswap32(load4(tq2 + a0, 0u));
      uint32_t cc, ff, rcc, rff;
      codes_flags4(c, cc, ff);
      codes_flags4(rc, rcc, rff);
      if (x0 < L1) {
        *(uint32_t *)(S1 + x0) = c;
        *(uint32_t *)(Q1 + x0) = q;
        ((uint8_t *)S1c)[x0 >> 2] = (uint8_t)cc;
        ((uint8_t *)S1f)[x0 >> 2] = (uint8_t)ff;
      }
      if (x0 < L2) {  // RC[j] = comp(s2[L2 - 1 - j]), RQ[j] = tq2[L2 - 1 - j]
        *(uint32_t *)(RC + x0) = rc;
        *(uint32_t *)(RQ + x0) = rq;
        ((uint8_t *)RCc)[x0 >> 2] = (uint8_t)rcc;
        ((uint8_t *)RCf)[x0 >> 2] = (uint8_t)rff;
      }
      const uint32_t v1 = x0 >= L1 ? 0u : L1 - x0 >= 4 ? ~0u : (1u << (8 * (L1 - x0))) - 1u;
      const uint32_t v2 = x0 >= L2 ? 0u : L2 - x0 >= 4 ? ~0u : (1u << (8 * (L2 - x0))) - 1u;
      bad2 |= (zero_bytes(rc) & v2) != 0;
      hasN |= ((eq_bytes(c, 0x4e4e4e4eu) & v1) | (eq_bytes(rc, 0x4e4e4e4eu) & v2)) != 0;
    }
    wave_sync_lds();
    if (__ballot(bad2)) {
      if (lane == 0) fq_fail(err, 2 * p + 1, FQ_E_CHAR2);
      continue;
    }
    hasN = __ballot(hasN) != 0;
    const int16_t len = (int16_t)(L2 < L1 ? L2 : L1);
    const int16_t start_i = (len == (int16_t)L1) ? 0 : (int16_t)(L1 - len);
    const int n_off = len - MIN_OVERLAP + EXTRA_TEST_OVERLAP;  // offsets i in [0, n_off)
    int16_t found_i = -1, best_i = -1;
    bool abort_merge = false, qbad = false, stop = false;
    for (int r0 = 0; r0 < n_off && !stop; r0 += 64) {
      // 1. fast filter of offsets r0 .. r0 + 63
      const int i = r0 + lane;
      // every lane runs the same steps (a uniform exit on a ballot, no per-lane loop masks): a lane past the
      // offsets or already over its limit keeps adding masked or surplus counts, which change no verdict
      const bool live = i < n_off;
      const int ov = live ? len - i : 0;
      const int emax = (MAX_MISMATCHES + (EXTRA_PER_1000 * ov / 1000)) * 4 / 3 + 1;
      // 32 bases per step: mate 1 from base start_i + i on (funnels of two code and two flag words) against
      // mate 2's; a base differs when its code or its flag does
      const int b0 = 2 * (start_i + (live ? i : 0)), k0 = b0 >> 6, sh = b0 & 63;
      int mm = 0;
      for (int j = 0; __ballot(j < ov && mm <= emax) != 0; j += 32) {
        const int k = k0 + (j >> 5);
        const uint64_t ca = (S1c[k] >> sh) | ((S1c[k + 1] << 1) << (63 - sh));
        const uint64_t fa = (S1f[k] >> sh) | ((S1f[k + 1] << 1) << (63 - sh));
        uint64_t x = (ca ^ RCc[j >> 5]) | (fa ^ RCf[j >> 5]);
        x = (x | (x >> 1)) & 0x5555555555555555ull;
        const int left = ov - j;  // bases of this step inside the overlap
        x &= left >= 32 ? ~0ull : left > 0 ? (1ull << (2 * left)) - 1 : 0ull;
        mm += __popcll(x);
      }
      const bool pass = live && mm <= emax;
      uint64_t kept = __ballot(pass);
      // 2. + 3. the kept offsets in order
      while (kept && !stop) {
        const int io = r0 + __ffsll((long long)kept) - 1;
        kept &= kept - 1;
        const int16_t overlap = len - (int16_t)io;
        const int16_t this_max = MAX_MISMATCHES + (EXTRA_PER_1000 * overlap / 1000);
        const int16_t err_max = this_max * 4 / 3 + 1;
        const int base = start_i + io;
        uint32_t cM = 0, cN = 0, cB = 0, matches = 0;
        int jb = -1, ev = 0;  // break position; 1 too many mismatches, 2 abort (N rules), 3 bad quality
        double perror = 0.0;
        for (int c0 = 0; c0 < overlap && jb < 0; c0 += 64) {
          const int j = c0 + lane;
          const bool in = j < overlap;
          if (!hasN) {  // (uniform) a pair without N: no both-N or N-mismatch terms, no quality effects
            const char ps = in ? S1[base + j] : 'A', rs = in ? RC[j] : 'A';
            const bool eq = in && ps == rs, mis = in && ps != rs;
            const uint8_t qa = in ? (uint8_t)(Q1[base + j] - qual_offset) : 0;
            const uint8_t qb = in ? (uint8_t)(RQ[j] - qual_offset) : 0;
            const bool bq = mis && (qa >= 81 || qb >= 81);
            const uint64_t bmis = __ballot(mis);
            const uint32_t M = cM + lanes_below(bmis) + mis;
            const int e = !in ? 0 : bq ? 3 : (int)M > err_max ? 1 : 0;
            const uint64_t evm = __ballot(e != 0);
            const int f = evm ? __ffsll((long long)evm) - 1 : 64;
            const uint64_t upto = f < 64 ? (f == 63 ? ~0ull : ((2ull << f) - 1)) : ~0ull;  // lanes <= f
            matches += (uint32_t)__popcll(__ballot(eq) & upto);
            double t2 = 0.0;
            if (mis && !bq) {
              const uint8_t dq = qa > qb ? qa - qb : qb - qa;
              t2 = dq <= 2 ? 0.5 : q2p[dq];
            }
            uint64_t mm = __ballot(mis && !bq) & upto;
            while (mm) {
              const int l = __ffsll((long long)mm) - 1;
              mm &= mm - 1;
              perror += lane_f64(t2, l);
            }
            if (f < 64) {
              jb = c0 + f;
              ev = (int)lane_u32((uint32_t)e, f);
              cM = lane_u32(M, f);
            } else {
              cM += (uint32_t)__popcll(bmis);
            }
            continue;
          }
          const char ps = in ? S1[base + j] : 'A', rs = in ? RC[j] : 'A';
          const bool eq = in && ps == rs, both = eq && ps == 'N', mis = in && ps != rs;
          const bool nmis = mis && (ps == 'N' || rs == 'N');
          const uint8_t qa = (ps == 'N' || !in) ? 0 : (uint8_t)(Q1[base + j] - qual_offset);
          const uint8_t qb = (rs == 'N' || !in) ? 0 : (uint8_t)(RQ[j] - qual_offset);
          const bool bq = mis && (qa >= 81 || qb >= 81);
          // the running counts up to j from ballots: mismatches (+1 more at an N), N bases (2 at a both-N),
          // both-N positions; v_mbcnt counts a mask's lanes below this one
          const uint64_t bmis = __ballot(mis), bnm = __ballot(nmis), bboth = __ballot(both);
          const uint32_t im = lanes_below(bmis) + mis, in_ = lanes_below(bnm) + nmis, ib = lanes_below(bboth) + both;
          const uint32_t M = cM + im + in_, NC = cN + 2 * ib + in_, B = cB + ib;
          // the reference's checks at j, in its order: a second both-N (in the match branch), a bad quality (in
          // the mismatch branch), then more than 3 N, then too many mismatches
          const int e = !in ? 0 : (both && B >= 2) ? 2 : bq ? 3 : NC > 3 ? 2 : (int)M > err_max ? 1 : 0;
          const uint64_t evm = __ballot(e != 0);
          const int f = evm ? __ffsll((long long)evm) - 1 : 64;
          const uint64_t upto = f < 64 ? (f == 63 ? ~0ull : ((2ull << f) - 1)) : ~0ull;  // lanes <= f
          matches += (uint32_t)__popcll(__ballot(eq) & upto);
          // the error-probability sum, mismatch by mismatch in order
          double t1 = 0.0, t2 = 0.0;
          if (mis && !bq) {
            t1 = ps == 'N' ? q2p[qb] : rs == 'N' ? q2p[qa] : 0.0;
            const uint8_t dq = qa > qb ? qa - qb : qb - qa;
            t2 = dq <= 2 ? 0.5 : q2p[dq];
          }
          uint64_t mm = __ballot(mis && !bq) & upto;
          const uint64_t nm = bnm;
          while (mm) {
            const int l = __ffsll((long long)mm) - 1;
            mm &= mm - 1;
            if ((nm >> l) & 1ull) perror += lane_f64(t1, l);
            perror += lane_f64(t2, l);
          }
          // the scan's quality effects (an N's quality := the offset), in LDS for the output
          if (nmis && j <= c0 + f) {
            if (ps == 'N')
              Q1[base + j] = (char)qual_offset;
            else
              RQ[j] = (char)qual_offset;
          }
          if (f < 64) {
            jb = c0 + f;
            ev = (int)lane_u32((uint32_t)e, f);
            cM = lane_u32(M, f);
          } else {
            const uint32_t pm = (uint32_t)__popcll(bmis), pn = (uint32_t)__popcll(bnm), pb = (uint32_t)__popcll(bboth);
            cM += pm + pn;
            cN += 2 * pb + pn;
            cB += pb;
          }
        }
        wave_sync_lds();
        if (ev == 3) {
          qbad = true;
          stop = true;
          break;
        }
        const int16_t checked = jb >= 0 ? (int16_t)(jb + 1) : overlap;
        const int16_t mismatches = (int16_t)cM;
        if (ev == 2) {
          abort_merge = true;
          ambiguous++;
        }
        int16_t match_thres = overlap - this_max;
        if (match_thres < MIN_OVERLAP) match_thres = MIN_OVERLAP;
        if ((int16_t)matches >= match_thres && checked == overlap && mismatches <= this_max &&
            perror / overlap <= MAX_PERROR) {
          if (best_i < 0 && found_i < 0) {
            best_i = (int16_t)io;
          } else {
            ambiguous++;
            best_i = -1;
            stop = true;
          }
        } else if (checked == overlap && mismatches <= err_max && perror / overlap <= MAX_PERROR * 4 / 3) {
          found_i = (int16_t)io;
          if (best_i >= 0) {
            ambiguous++;
            best_i = -1;
            stop = true;
          }
        }
        if (abort_merge) stop = true;  // the next offset's "if (abort_merge) break"
      }
    }
    if (qbad) {
      if (lane == 0) fq_fail(err, 2 * p + 1, FQ_E_QUAL);
      continue;
    }
    uint32_t info = hasN ? MP_HASN : 0u;
    if (best_i >= 0 && !abort_merge) {
      const int ov = len - best_i;
      info |= (uint32_t)ov + 1u;
      if (lane == 0) {
        out_len[2 * p] = (unsigned long long)(L1 + L2 - ov);
        out_len[2 * p + 1] = 1;
      }
      merged++;
      ov_bases += (uint64_t)ov;
    } else if (lane == 0) {
      out_len[2 * p] = (unsigned long long)L1;
      out_len[2 * p + 1] = (unsigned long long)L2;
    }
    if (lane == 0) pair_info[p] = info;
    if (hasN) {  // the qualities as the scan left them, for k_fq_merge_pack
      char *cq1 = scratch + rec_offs[2 * p], *crq2 = scratch + rec_offs[2 * p + 1];
      for (int x = lane; x < L1; x += 64) cq1[x] = Q1[x];
      for (int j = lane; j < L2; j += 64) crq2[j] = RQ[j];
    }
    wave_sync_lds();  // the next pair overwrites the wave's LDS
  }
  if (lane == 0 && (merged | ambiguous)) {
    atomicAdd(&stats[1], (unsigned long long)merged);
    atomicAdd(&stats[2], (unsigned long long)ambiguous);
    atomicAdd(&stats[3], (unsigned long long)ov_bases);
  }
}

// Writes a wave's 256 packed bytes of one record (lane t: record bytes base + 4t .. + 3, packed in w) as ALIGNED
// dwords, like k_fq_pack: the output dword of lane t holds record bytes [base + 4t - s, base + 4t + 4 - s), s the
// record's misalignment, i.e. the high s bytes of the next lower lane's word (wave_shr:1 DPP; lane 0 takes the
// previous step's lane 63, carry) and the low 4 - s of its own. Only the record's first and last dwords, which it
// shares with its neighbours, are written bytewise. Every lane of the wave must call it (the DPP move).
__device__ __forceinline__ void put_run(uint8_t *dst, int L, int base, int lane, uint32_t w, uint32_t &carry) {
  const int s = (int)((uintptr_t)dst & 3u);
  const uint32_t wm = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)w, 0x138, 0xf, 0xf, false);
  carry = (uint32_t)__builtin_amdgcn_readlane((int)w, 63);
  const uint32_t ow = s ? __builtin_amdgcn_alignbyte(w, wm, 4 - s) : w;
  const int x0 = base + 4 * lane - s;  // record byte of the output dword's first byte
  uint8_t *const o = dst + x0;          // aligned
  if (x0 >= 0 && x0 + 4 <= L) {
    *(uint32_t *)o = ow;
  } else if (x0 < L && x0 + 4 > 0) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (x0 + j >= 0 && x0 + j < L) o[j] = (uint8_t)(ow >> (8 * j));
  }
}

// One wave per pair (grid-stride), four output bytes per lane and step: the pair's output reads from its
// descriptor in one round of loads. Merged read (x < L1 - ov: mate 1; the overlap: the higher-quality base,
// :449-469; then the rest of mate 2 reverse-complemented, :472-473) + the dummy "N", or both mates as read.
// The merge rules run per byte as selects, the four bytes are packed by pack4 (k_fq_pack's SWAR path) and
// stored as aligned dwords (put_run).
__global__ __launch_bounds__(64 * MG_WAVES) void k_fq_merge_pack(const char *text, const PairDesc *desc, uint64_t n_pairs,
                                                                  const unsigned long long *rec_offs,
                                                                  const char *scratch, const uint32_t *pair_info,
                                                                  const unsigned long long *out_offs, int qual_offset,
                                                                  uint8_t *out, unsigned long long *err) {
  // the wave index as a scalar: the pair index, its descriptor, verdict and offsets then live in scalar registers
  // (scalar loads), not in 25 VGPRs of every lane
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int max_match_qual = 41 + qual_offset;
  const uint64_t stride = (uint64_t)gridDim.x * MG_WAVES;
  // The next pair's descriptor, verdict and offsets are loaded while this pair is packed: the text loads of a
  // pair are then its only global round trip before the stores.
  uint64_t p = (uint64_t)blockIdx.x * MG_WAVES + w;
  PairDesc dn{0, 0, 0, 0, ~0u, 0};
  uint32_t infon = 0;
  unsigned long long ro0n = 0, ro1n = 0, oo0n = 0, oo1n = 0;
  if (p < n_pairs) {
    dn = desc[p];
    infon = pair_info[p];
    ro0n = rec_offs[2 * p];
    ro1n = rec_offs[2 * p + 1];
    oo0n = out_offs[2 * p];
    oo1n = out_offs[2 * p + 1];
  }
  for (; p < n_pairs; p += stride) {
    const PairDesc d = dn;
    const uint32_t info = infon;
    const unsigned long long ro0 = ro0n, ro1 = ro1n, oo0 = oo0n, oo1 = oo1n;
    const uint64_t pn = p + stride;
    if (pn < n_pairs) {
      dn = desc[pn];
      infon = pair_info[pn];
      ro0n = rec_offs[2 * pn];
      ro1n = rec_offs[2 * pn + 1];
      oo0n = out_offs[2 * pn];
      oo1n = out_offs[2 * pn + 1];
    }
    if (d.L1 == ~0u) continue;
    const int ov = (int)(info & ~MP_HASN) - 1;  // -1: not merged
    const bool hasN = (info & MP_HASN) != 0;
    const int L1 = (int)d.L1, L2 = (int)d.L2;
    const char *s1 = text + d.s1, *tq1 = text + d.q1, *s2 = text + d.s2, *tq2 = text + d.q2;
    const char *cq1 = scratch + ro0, *crq2 = scratch + ro1;
    uint8_t *dst0 = out + oo0, *dst1 = out + oo1;
    const int Lo0 = ov >= 0 ? L1 + L2 - ov : L1, st = ov >= 0 ? L1 - ov : L1;
    bool bad = false;
    uint32_t carry = 0;
    const int s0 = (int)((uintptr_t)dst0 & 3u);
    for (int base = 0; base - s0 < Lo0; base += 256) {
      const int x0 = base + 4 * lane;
      // branch-free: every lane loads (addresses clamped into the lines) and computes, selects pick the result
      const int xs = min(x0, L1 - 1);
      const uint32_t cs0 = load4(s1 + xs, 0u), cq0 = load4((hasN ? cq1 : tq1) + xs, 0u);
      const uint32_t cs = x0 < L1 ? cs0 : 0u, cq = x0 < L1 ? cq0 : 0u;
      const int jj = min(max(x0 - st, -3), L2 - 1);  // RC index of output byte x0 (clamped)
      const uint32_t rc = comp4(__builtin_bswap32(load4(s2 + (L2 - 4 - jj), 0u)));
      // (the scratch copy is in RC order; before its start, shift instead of reading before the buffer)
      const uint32_t rq = hasN ? (jj >= 0 ? load4(crq2 + jj, 0u) : load4(crq2, 0u) << (8 * -jj))
                               : __builtin_bswap32(load4(tq2 + (L2 - 4 - jj), 0u));
      uint32_t mc = 0, mq = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int x = x0 + i;
        const char c = (char)(cs >> (8 * i)), q = (char)(cq >> (8 * i));
        const char r = (char)(rc >> (8 * i)), rqq = (char)(rq >> (8 * i));
        // :449-469 in the overlap (both bases), :472-473 after it (mate 2's)
        const uint16_t nq1 = (uint16_t)(q + rqq - qual_offset);
        const char qeq = (char)(nq1 > max_match_qual ? max_match_qual : nq1);
        const bool lt = q < rqq;
        const uint8_t nq2 = (uint8_t)(lt ? rqq - q + qual_offset : q - rqq + qual_offset);
        const char qne = (char)(nq2 > 2 + qual_offset ? nq2 : 2 + qual_offset);
        const bool inB = x >= st && x < L1, inC = x >= L1;
        const char co = inB ? (c == r ? c : (lt ? r : c)) : inC ? r : c;
        const char qo = inB ? (c == r ? qeq : qne) : inC ? rqq : q;
        mc |= (uint32_t)(uint8_t)co << (8 * i);
        mq |= (uint32_t)(uint8_t)qo << (8 * i);
      }
      const bool mrg = ov >= 0 && x0 + 3 >= st;
      bool bw = false;
      const uint32_t pw = pack4(mrg ? mc : cs, mrg ? mq : cq, max(1, min(4, Lo0 - x0)), qual_offset, bw);
      const uint32_t w = x0 < Lo0 ? pw : 0u;
      bad |= bw && x0 < Lo0;
      put_run(dst0, Lo0, base, lane, w, carry);
    }
    if (ov >= 0) {
      if (lane == 0) dst1[0] = 4;  // the dummy mate "N" with quality qual_offset
    } else {
      // mate 2 as read (its bases passed the revcomp check)
      const int s1o = (int)((uintptr_t)dst1 & 3u);
      carry = 0;
      for (int base = 0; base - s1o < L2; base += 256) {
        const int x0 = base + 4 * lane;
        uint32_t w = 0;
        bool bb = false;
        if (x0 < L2) w = pack4(load4(s2 + x0, 0u), load4(tq2 + x0, 0u), min(4, L2 - x0), qual_offset, bb);
        put_run(dst1, L2, base, lane, w, carry);
      }
    }
    if (__ballot(bad) && lane == 0) fq_fail(err, 2 * p + 1, FQ_E_CHAR1);  // mate 1's (or the merged) PackedRead
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

size_t fq_pair_desc_bytes(uint64_t n_pairs) {  // the descriptors, then the long-pair counter and list
  return (((size_t)n_pairs * sizeof(PairDesc) + 63) & ~(size_t)63) + 64 + (size_t)n_pairs * 4 + 64;
}

hipError_t launch_fq_pair_records(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_rec,
                                  unsigned long long *len, unsigned long long *err, void *desc_buf, hipStream_t s) {
  const uint64_t n_pairs = n_rec / 2;
  hipError_t e = hipMemsetAsync(long_pairs(desc_buf, n_pairs), 0, 4, s);
  if (e != hipSuccess) return e;
  const uint64_t nt = n_rec / 2 + 1;
  k_fq_pair_records<<<dim3((unsigned)((nt + FQ_THREADS - 1) / FQ_THREADS)), dim3(FQ_THREADS), 0, s>>>(
      text, n, line_end, n_rec, len, err, (PairDesc *)desc_buf, long_pairs(desc_buf, n_pairs));
  return hipGetLastError();
}

hipError_t launch_fq_merge(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_pairs,
                           const unsigned long long *rec_offs, int qual_offset, char *scratch, void *desc_buf,
                           uint32_t *pair_info, unsigned long long *out_len, unsigned long long *err,
                           unsigned long long *stats, hipStream_t s) {
  // (the descriptors and the long-pair list come from launch_fq_pair_records)
  PairDesc *desc = (PairDesc *)desc_buf;
  uint32_t *long_list = long_pairs(desc_buf, n_pairs);
  hipError_t e = hipSuccess;
  // grid-stride over the pairs, one wave each; enough waves to fill the chip several times over
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((n_pairs + MG_WAVES - 1) / MG_WAVES, 16384));
  k_fq_merge<MG_SHORT><<<dim3((unsigned)blocks), dim3(64 * MG_WAVES), 0, s>>>(
      text, desc, n_pairs, rec_offs, qual_offset, scratch, pair_info, out_len, err, stats, nullptr);
  if ((e = hipGetLastError()) != hipSuccess || MG_SHORT >= MG_MAXL) return e;
  // the listed long pairs (the waves of an empty list exit at once)
  k_fq_merge<MG_MAXL><<<dim3((unsigned)std::min<uint64_t>(blocks, 1024)), dim3(64 * MG_WAVES), 0, s>>>(
      text, desc, n_pairs, rec_offs, qual_offset, scratch, pair_info, out_len, err, stats, long_list);
  return hipGetLastError();
}

hipError_t launch_fq_merge_pack(const char *text, const void *desc_buf, uint64_t n_pairs,
                                const unsigned long long *rec_offs, const char *scratch, const uint32_t *pair_info,
                                const unsigned long long *out_offs, int qual_offset, uint8_t *out,
                                unsigned long long *err, hipStream_t s) {
  if (!n_pairs) return hipSuccess;
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((n_pairs + MG_WAVES - 1) / MG_WAVES, 16384));
  k_fq_merge_pack<<<dim3((unsigned)blocks), dim3(64 * MG_WAVES), 0, s>>>(
      text, (const PairDesc *)desc_buf, n_pairs, rec_offs, scratch, pair_info, out_offs, qual_offset, out, err);
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

// dst[i] = src[i] + delta (the offsets of one block's PackedReads appended to a file's; mhmkc_add_fastq_file)
__global__ __launch_bounds__(256) void k_offs_rebase(unsigned long long *dst, const unsigned long long *src, uint64_t n,
                                                     unsigned long long delta) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i] + delta;
}

hipError_t launch_offs_rebase(unsigned long long *dst, const unsigned long long *src, uint64_t n, unsigned long long delta,
                              hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>(4096, (n + 255) / 256);
  k_offs_rebase<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(dst, src, n, delta);
  return hipGetLastError();
}

}  // namespace mhm
