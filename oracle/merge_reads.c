/* TEST INFRASTRUCTURE ONLY (never linked into libmhmkc): plain-C restatement of the reference's read-pair
 * merging, merge_reads (src/merge_reads.cpp:237-588), for one interleaved paired FASTQ text, followed by the
 * PackedRead constructor (src/packed_reads.cpp:73-109) of every read it adds to packed_reads_list.
 *
 * Per pair (records 2p and 2p+1, FastqReader::get_next_fq_record :504-551 parses them, interleaving a pair
 * of files the same way):
 *   - the normalized names (get_fq_name :73-122, then replace_spaces) must agree but for their last two
 *     characters, and end in '1' and '2' (:320-321, DIE otherwise);
 *   - rc_seq2 = revcomp(seq2) (utils.cpp: IUPAC -> N), rev_quals2 = reversed quals2;
 *   - offsets i of rc_seq2 against seq1 are scanned in order (:345-444): a fast mismatch count
 *     (fast_count_mismatches :183-230) skips offsets with more than error_max_mismatch mismatches; the others
 *     are checked base by base with the N rules (both-N twice or more than 3 N: abort; an N zeroes its own
 *     quality, in quals1 or rev_quals2), the differential-quality error sum and the break on too many
 *     mismatches; a good offset is kept if it is the first good or weak one, a second good or a good after a
 *     weak one (or a weak after a good) makes the pair ambiguous;
 *   - a kept offset merges (:446-486): per overlapped base the higher-quality base, qualities added on a match
 *     (capped at 41 + offset) or differenced on a mismatch (floored at 2 + offset), then the rest of rc_seq2;
 *     the merged read is added with a dummy mate "N"; otherwise both mates are added as read (:487-491), with
 *     quals1 as the scan left it.
 * A record 2p without a mate ends the file (:315-317). Nothing here was copied from the reference; it is a
 * restatement of the cited lines. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Q2Perror of merge_reads.cpp:73-81: 10^(-q/10) as the reference tabulates it (81 entries, q = 0..80) */
static const double Q2P[81] = {
    1.0,       0.7943,    0.6309,    0.5012,    0.3981,    0.3162,    0.2512,    0.1995,    0.1585,    0.1259,     0.1,
    0.07943,   0.06310,   0.05012,   0.03981,   0.03162,   0.02512,   0.01995,   0.01585,   0.01259,   0.01,       0.007943,
    0.006310,  0.005012,  0.003981,  0.003162,  0.002512,  0.001995,  0.001585,  0.001259,  0.001,     0.0007943,  0.0006310,
    0.0005012, 0.0003981, 0.0003162, 0.0002512, 0.0001995, 0.0001585, 0.0001259, 0.0001,    7.943e-05, 6.310e-05,  5.012e-05,
    3.981e-05, 3.162e-05, 2.512e-05, 1.995e-05, 1.585e-05, 1.259e-05, 1e-05,     7.943e-06, 6.310e-06, 5.012e-06,  3.981e-06,
    3.162e-06, 2.512e-06, 1.995e-06, 1.585e-06, 1.259e-06, 1e-06,     7.943e-07, 6.310e-07, 5.012e-07, 3.981e-07,  3.1622e-07,
    2.512e-07, 1.995e-07, 1.585e-07, 1.259e-07, 1e-07,     7.943e-08, 6.310e-08, 5.012e-08, 3.981e-08, 3.1622e-08, 2.512e-08,
    1.995e-08, 1.585e-08, 1.259e-08, 1e-08};

static int mr_isspace(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
static uint64_t mr_rtrim(const char *s, uint64_t b, uint64_t e) {
  while (e > b && mr_isspace((unsigned char)s[e - 1])) e--;
  return e;
}

/* get_fq_name's normalized name of the trimmed id line [b, e) as (prefix [pb, pe) of the text, last char),
 * where the full normalized name is prefix + one separator character + last (or the header itself);
 * returns 0 for an unknown format. */
static int mr_name(const char *s, uint64_t b, uint64_t e, uint64_t *pb, uint64_t *pe, char *last) {
  const char *h = s + b + 1;
  const uint64_t len = mr_rtrim(s, b + 1, e) - (b + 1);
  *pb = b + 1;
  if (len >= 3 && h[len - 2] != '/') {
    if (h[len - 2] == 'R') { /* pair-R1 -> pair/1 */
      *pe = b + 1 + len - 3;
      *last = h[len - 1];
      return 1;
    }
    uint64_t ep = len;
    for (uint64_t i = 0; i < len; i++)
      if (h[i] == '\t') { ep = i; break; }
    if (ep == len) {
      for (uint64_t i = 0; i < len; i++)
        if (h[i] == ' ') { ep = i; break; }
      if (ep == len) { /* no comment: unchanged */
        *pe = b + 1 + (len >= 2 ? len - 2 : 0);
        *last = len ? h[len - 1] : 0;
        return 1;
      }
    }
    if (ep > 3 && h[ep - 2] == '/' && (h[ep - 1] == '1' || h[ep - 1] == '2')) { /* truncated at the comment */
      *pe = b + 1 + ep - 2;
      *last = h[ep - 1];
      return 1;
    }
    if (len < ep + 7 || h[ep + 2] != ':' || h[ep + 4] != ':' || h[ep + 6] != ':' || (h[ep + 1] != '1' && h[ep + 1] != '2'))
      return 0;
    *pe = b + 1 + ep; /* pair 1:N:... -> pair/1 */
    *last = h[ep + 1];
    return 1;
  }
  *pe = b + 1 + (len >= 2 ? len - 2 : 0);
  *last = len ? h[len - 1] : 0;
  return 1;
}

static int mr_same_prefix(const char *s, uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1) {
  if (a1 - a0 != b1 - b0) return 0;
  for (uint64_t i = 0; i < a1 - a0; i++) {
    char x = s[a0 + i], y = s[b0 + i];
    if (x == ' ') x = '_'; /* replace_spaces */
    if (y == ' ') y = '_';
    if (x != y) return 0;
  }
  return 1;
}

static char mr_comp(char c) { /* revcomp (utils.cpp): complement, IUPAC -> N; anything else DIEs */
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    case 'N': case 'U': case 'R': case 'Y': case 'K': case 'M': case 'S': case 'W': case 'B': case 'D': case 'H':
    case 'V': return 'N';
  }
  return 0;
}

static int mr_code(char c) { /* PackedRead::PackedRead */
  switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'N': case 'U': case 'R': case 'Y': case 'K': case 'M': case 'S': case 'W': case 'B': case 'D': case 'H':
    case 'V': return 4;
  }
  return -1;
}

static int mr_pack(const char *seq, const char *q, int64_t L, int off, uint8_t *out) {
  for (int64_t i = 0; i < L; i++) {
    const int c = mr_code(seq[i]);
    if (c < 0) return -1;
    int v = (int)(signed char)q[i] - off;
    if (v > 31) v = 31;
    out[i] = (uint8_t)(c | (uint8_t)((unsigned char)v << 3));
  }
  return 0;
}

/* Error kinds (returned negated): 1..7 as orc_fastq_pack, 8 mismatched pair names, 9 mismatched pair numbers,
 * 10 invalid quality in an overlap (the :409-413 DIE). stats: [pairs, merged, ambiguous, overlap bases]. */
int64_t orc_merge_fastq(const char *text, uint64_t n, int qual_offset, uint8_t *out, uint64_t *offs, uint64_t *stats,
                        uint64_t *err_rec) {
  const int16_t MIN_OVERLAP = 12, EXTRA_TEST_OVERLAP = 2, MAX_MISMATCHES = 3, EXTRA_PER_1000 = 150;
  const double MAX_PERROR = 0.025;
  const int max_match_qual = 41 + qual_offset;
  uint64_t pos = 0, rec = 0, nr = 0, nb = 0;
  offs[0] = 0;
  memset(stats, 0, 4 * sizeof(uint64_t));
  char *s1 = NULL, *q1 = NULL, *rc2 = NULL, *rq2 = NULL;
  int64_t cap = 0;
  int64_t ret = 0;
  for (;;) {
    uint64_t lb[2][4], le[2][4], te[2][4];
    int got = 0;
    for (int m = 0; m < 2; m++) {
      if (pos >= n) break;
      for (int i = 0; i < 4; i++) {
        if (pos >= n) { *err_rec = rec + m; ret = -7; goto done; }
        const char *nl = memchr(text + pos, '\n', n - pos);
        const uint64_t end = nl ? (uint64_t)(nl - text) : n;
        lb[m][i] = pos;
        le[m][i] = end;
        te[m][i] = mr_rtrim(text, pos, end);
        pos = end + 1;
      }
      for (int i = 0; i < 4; i++)
        if (le[m][i] - lb[m][i] > 2045) { *err_rec = rec + m; ret = -5; goto done; }
      if (te[m][0] == lb[m][0] || text[lb[m][0]] != '@') { *err_rec = rec + m; ret = -1; goto done; }
      if (le[m][2] == lb[m][2] || text[lb[m][2]] != '+') { *err_rec = rec + m; ret = -2; goto done; }
      uint64_t pb, pe;
      char last;
      if (!mr_name(text, lb[m][0], te[m][0], &pb, &pe, &last)) { *err_rec = rec + m; ret = -3; goto done; }
      if (te[m][1] - lb[m][1] != te[m][3] - lb[m][3]) { *err_rec = rec + m; ret = -4; goto done; }
      got++;
    }
    if (got < 2) break; /* no record, or a last record without its mate: the merge loop stops (:315-317) */
    {
      uint64_t pb1, pe1, pb2, pe2;
      char l1, l2;
      mr_name(text, lb[0][0], te[0][0], &pb1, &pe1, &l1);
      mr_name(text, lb[1][0], te[1][0], &pb2, &pe2, &l2);
      if (!mr_same_prefix(text, pb1, pe1, pb2, pe2)) { *err_rec = rec; ret = -8; goto done; }
      if (l1 != '1' || l2 != '2') { *err_rec = rec; ret = -9; goto done; }
    }
    const int64_t L1 = (int64_t)(te[0][1] - lb[0][1]), L2 = (int64_t)(te[1][1] - lb[1][1]);
    if (L1 + L2 + 2 > cap) {
      cap = 2 * (L1 + L2 + 2);
      s1 = realloc(s1, cap);
      q1 = realloc(q1, cap);
      rc2 = realloc(rc2, cap);
      rq2 = realloc(rq2, cap);
    }
    memcpy(s1, text + lb[0][1], L1);
    memcpy(q1, text + lb[0][3], L1);
    for (int64_t j = 0; j < L2; j++) {
      rc2[j] = mr_comp(text[lb[1][1] + L2 - 1 - j]);
      if (!rc2[j]) { *err_rec = rec + 1; ret = -6; goto done; }
      rq2[j] = text[lb[1][3] + L2 - 1 - j];
    }
    stats[0]++;
    int abort_merge = 0;
    const int16_t len = (int16_t)(L2 < L1 ? L2 : L1);
    const int16_t start_i = (len == (int16_t)L1) ? 0 : (int16_t)(L1 - len);
    int16_t found_i = -1, best_i = -1;
    for (int16_t i = 0; i < len - MIN_OVERLAP + EXTRA_TEST_OVERLAP; i++) {
      if (abort_merge) break;
      const int16_t overlap = len - i;
      const int16_t this_max = MAX_MISMATCHES + (EXTRA_PER_1000 * overlap / 1000);
      const int16_t err_max = this_max * 4 / 3 + 1;
      int16_t fast = 0;
      for (int16_t j = 0; j < overlap && fast <= err_max; j++) fast += s1[start_i + i + j] != rc2[j];
      if (fast > err_max) continue;
      int16_t matches = 0, mismatches = 0, bothNs = 0, Ncount = 0, checked = 0;
      double perror = 0.0;
      for (int16_t j = 0; j < overlap; j++) {
        checked++;
        const int p = start_i + i + j;
        const char ps = s1[p], rs = rc2[j];
        if (ps == rs) {
          matches++;
          if (ps == 'N') {
            Ncount += 2;
            if (bothNs++) {
              abort_merge++;
              stats[2]++;
              break;
            }
          }
        } else {
          mismatches++;
          /* the quality DIE of :409-413 comes after the N branch in the reference, whose table read is then
           * out of range for the same bad quality; checking first gives the same outcome without it */
          if (ps == 'N') {
            mismatches++;
            Ncount++;
            q1[p] = (char)qual_offset;
          } else if (rs == 'N') {
            Ncount++;
            mismatches++;
            rq2[j] = (char)qual_offset;
          }
          const uint8_t a = (uint8_t)(q1[p] - qual_offset), b = (uint8_t)(rq2[j] - qual_offset);
          if (a >= 81 || b >= 81) { *err_rec = rec; ret = -10; goto done; }
          if (ps == 'N')
            perror += Q2P[b];
          else if (rs == 'N')
            perror += Q2P[a];
          const uint8_t dq = a > b ? a - b : b - a;
          perror += dq <= 2 ? 0.5 : Q2P[dq];
        }
        if (Ncount > 3) {
          abort_merge++;
          stats[2]++;
          break;
        }
        if (mismatches > err_max) break;
      }
      int16_t match_thres = overlap - this_max;
      if (match_thres < MIN_OVERLAP) match_thres = MIN_OVERLAP;
      if (matches >= match_thres && checked == overlap && mismatches <= this_max && perror / overlap <= MAX_PERROR) {
        if (best_i < 0 && found_i < 0) {
          best_i = i;
        } else {
          stats[2]++;
          best_i = -1;
          break;
        }
      } else if (checked == overlap && mismatches <= err_max && perror / overlap <= MAX_PERROR * 4 / 3) {
        found_i = i;
        if (best_i >= 0) {
          stats[2]++;
          best_i = -1;
          break;
        }
      }
    }
    uint8_t *o = out + nb;
    if (best_i >= 0 && !abort_merge) {
      const int16_t i = best_i, overlap = len - i;
      for (int16_t j = 0; j < overlap; j++) {
        const int p = start_i + i + j;
        if (s1[p] == rc2[j]) {
          const uint16_t nq = (uint16_t)(q1[p] + rq2[j] - qual_offset);
          q1[p] = (char)(nq > max_match_qual ? max_match_qual : nq);
        } else {
          uint8_t nq;
          if (q1[p] < rq2[j]) {
            nq = (uint8_t)(rq2[j] - q1[p] + qual_offset);
            s1[p] = rc2[j];
          } else {
            nq = (uint8_t)(q1[p] - rq2[j] + qual_offset);
          }
          q1[p] = (char)(nq > 2 + qual_offset ? nq : 2 + qual_offset);
        }
      }
      memcpy(s1 + L1, rc2 + overlap, L2 - overlap); /* seq1.substr(0, L1) + rc_seq2.substr(overlap) */
      memcpy(q1 + L1, rq2 + overlap, L2 - overlap);
      const int64_t Lm = L1 + L2 - overlap;
      if (mr_pack(s1, q1, Lm, qual_offset, o)) { *err_rec = rec; ret = -6; goto done; }
      const char nseq = 'N', nq = (char)qual_offset;
      mr_pack(&nseq, &nq, 1, qual_offset, o + Lm);
      nb += Lm + 1;
      offs[nr + 1] = nb - 1;
      offs[nr + 2] = nb;
      stats[1]++;
      stats[3] += overlap;
    } else {
      if (mr_pack(s1, q1, L1, qual_offset, o)) { *err_rec = rec; ret = -6; goto done; }
      if (mr_pack(text + lb[1][1], text + lb[1][3], L2, qual_offset, o + L1)) { *err_rec = rec + 1; ret = -6; goto done; }
      nb += L1 + L2;
      offs[nr + 1] = nb - L2;
      offs[nr + 2] = nb;
    }
    nr += 2;
    rec += 2;
  }
  ret = (int64_t)nr;
done:
  free(s1);
  free(q1);
  free(rc2);
  free(rq2);
  return ret;
}
