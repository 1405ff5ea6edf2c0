"""A second, independent restatement of merge_reads (src/merge_reads.cpp:237-588) at the string level, written
the way the reference code reads (std::string seq/quals, char arithmetic, the fast_count_mismatches helper as
a separate early-exit count), to cross-check the C oracle (oracle/merge_reads.c) on small inputs. TEST
INFRASTRUCTURE ONLY; slow (pure Python)."""
from __future__ import annotations

Q2PERROR = [
    1.0, 0.7943, 0.6309, 0.5012, 0.3981, 0.3162, 0.2512, 0.1995, 0.1585, 0.1259, 0.1,
    0.07943, 0.06310, 0.05012, 0.03981, 0.03162, 0.02512, 0.01995, 0.01585, 0.01259, 0.01, 0.007943,
    0.006310, 0.005012, 0.003981, 0.003162, 0.002512, 0.001995, 0.001585, 0.001259, 0.001, 0.0007943, 0.0006310,
    0.0005012, 0.0003981, 0.0003162, 0.0002512, 0.0001995, 0.0001585, 0.0001259, 0.0001, 7.943e-05, 6.310e-05, 5.012e-05,
    3.981e-05, 3.162e-05, 2.512e-05, 1.995e-05, 1.585e-05, 1.259e-05, 1e-05, 7.943e-06, 6.310e-06, 5.012e-06, 3.981e-06,
    3.162e-06, 2.512e-06, 1.995e-06, 1.585e-06, 1.259e-06, 1e-06, 7.943e-07, 6.310e-07, 5.012e-07, 3.981e-07, 3.1622e-07,
    2.512e-07, 1.995e-07, 1.585e-07, 1.259e-07, 1e-07, 7.943e-08, 6.310e-08, 5.012e-08, 3.981e-08, 3.1622e-08, 2.512e-08,
    1.995e-08, 1.585e-08, 1.259e-08, 1e-08]
COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}
COMP.update({c: "N" for c in "URYKMSWBDHV"})
CODE = {"A": 0, "C": 1, "G": 2, "T": 3}
CODE.update({c: 4 for c in "NURYKMSWBDHV"})


def records(text: str):
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    for r in range(0, len(lines) - 3, 4):
        yield [ln.rstrip() for ln in lines[r:r + 4]]


def norm_name(h: str) -> str:
    h = h[1:].rstrip()
    n = len(h)
    if n >= 3 and h[n - 2] != "/":
        if h[n - 2] == "R":
            return h[:n - 3] + "/" + h[n - 1]
        ep = h.find("\t")
        if ep < 0:
            ep = h.find(" ")
            if ep < 0:
                return h
        if ep > 3 and h[ep - 2] == "/" and h[ep - 1] in "12":
            return h[:ep]
        return h[:ep] + "/" + h[ep + 1]
    return h


def fast_count_mismatches(a: str, b: str, n: int, mx: int) -> int:
    mm = 0
    for j in range(n):
        mm += a[j] != b[j]
        if mm > mx:
            break
    return mm


def merge_pair(seq1, quals1, seq2, quals2, off):
    """-> (reads [(seq, quals)], merged, ambiguous_increments, overlap)"""
    quals1 = list(quals1)
    rc = "".join(COMP[c] for c in reversed(seq2))
    rq = list(reversed(quals2))
    seq1 = list(seq1)
    MIN_OVERLAP, EXTRA, MAXMM, PER1000, MAX_PERROR = 12, 2, 3, 150, 0.025
    amb = 0
    abort = 0
    ln = min(len(rc), len(seq1))
    start_i = 0 if ln == len(seq1) else len(seq1) - ln
    found_i = best_i = -1
    for i in range(ln - MIN_OVERLAP + EXTRA):
        if abort:
            break
        ov = ln - i
        tmax = MAXMM + (PER1000 * ov // 1000)
        emax = tmax * 4 // 3 + 1
        if fast_count_mismatches(seq1[start_i + i:], rc, ov, emax) > emax:
            continue
        matches = mism = both = ncount = checked = 0
        perror = 0.0
        for j in range(ov):
            checked += 1
            p = start_i + i + j
            ps, rs = seq1[p], rc[j]
            if ps == rs:
                matches += 1
                if ps == "N":
                    ncount += 2
                    both += 1
                    if both > 1:
                        abort += 1
                        amb += 1
                        break
            else:
                mism += 1
                if ps == "N":
                    mism += 1
                    ncount += 1
                    quals1[p] = chr(off)
                elif rs == "N":
                    ncount += 1
                    mism += 1
                    rq[j] = chr(off)
                q1, q2 = (ord(quals1[p]) - off) & 0xFF, (ord(rq[j]) - off) & 0xFF
                if q1 >= len(Q2PERROR) or q2 >= len(Q2PERROR):
                    raise ValueError("qual")
                if ps == "N":
                    perror += Q2PERROR[q2]
                elif rs == "N":
                    perror += Q2PERROR[q1]
                d = abs(q1 - q2)
                perror += 0.5 if d <= 2 else Q2PERROR[d]
            if ncount > 3:
                abort += 1
                amb += 1
                break
            if mism > emax:
                break
        thr = max(ov - tmax, MIN_OVERLAP)
        if matches >= thr and checked == ov and mism <= tmax and perror / ov <= MAX_PERROR:
            if best_i < 0 and found_i < 0:
                best_i = i
            else:
                amb += 1
                best_i = -1
                break
        elif checked == ov and mism <= emax and perror / ov <= MAX_PERROR * 4 / 3:
            found_i = i
            if best_i >= 0:
                amb += 1
                best_i = -1
                break
    if best_i >= 0 and not abort:
        ov = ln - best_i
        maxq = 41 + off
        for j in range(ov):
            p = start_i + best_i + j
            if seq1[p] == rc[j]:
                nq = ord(quals1[p]) + ord(rq[j]) - off
                quals1[p] = chr(min(nq, maxq))
            else:
                if ord(quals1[p]) < ord(rq[j]):
                    nq = (ord(rq[j]) - ord(quals1[p]) + off) & 0xFF
                    seq1[p] = rc[j]
                else:
                    nq = (ord(quals1[p]) - ord(rq[j]) + off) & 0xFF
                quals1[p] = chr(max(nq, 2 + off))
        s = "".join(seq1) + rc[ov:]
        q = "".join(quals1) + "".join(rq[ov:])
        return [(s, q), ("N", chr(off))], True, amb, ov
    return [("".join(seq1), "".join(quals1)), (seq2, quals2)], False, amb, 0


def pack(seq, quals, off):
    return bytes((CODE[c] | ((min(ord(q) - off, 31) & 0xFF) << 3) & 0xFF) for c, q in zip(seq, quals))


def merge_fastq(text: bytes, off: int = 33):
    recs = list(records(text.decode("latin-1")))
    out, offs = [], [0]
    st = {"pairs": 0, "merged": 0, "ambiguous": 0, "overlap_bases": 0}
    for p in range(0, len(recs) - 1, 2):
        (i1, s1, _, q1), (i2, s2, _, q2) = recs[p], recs[p + 1]
        n1, n2 = norm_name(i1).replace(" ", "_"), norm_name(i2).replace(" ", "_")
        assert n1[:-2] == n2[:-2] and n1[-1] == "1" and n2[-1] == "2", (n1, n2)
        st["pairs"] += 1
        reads, merged, amb, ov = merge_pair(s1, q1, s2, q2, off)
        st["merged"] += merged
        st["ambiguous"] += amb
        st["overlap_bases"] += ov
        for s, q in reads:
            out.append(pack(s, q, off))
            offs.append(offs[-1] + len(s))
    return b"".join(out), offs, st
