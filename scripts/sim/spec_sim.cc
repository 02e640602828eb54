// CPU simulation of the Zstd L1 speculative block-parallel parse (analysis
// only, not shipped): the fast parse of oracle/zstd_l1_oracle.c with its table
// reads instrumented.  Per round it reports how many blocks change and, for
// the "resume" idea, how much of each changed block must be parsed again: a
// block's parse is unchanged up to its first read of a bucket whose input
// value changed (or from the start if its repeat offsets changed).
//   g++ -O2 -o /tmp/spec_sim scripts/sim/spec_sim.cc && /tmp/spec_sim T 5 4194304
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include "../../juicefs_amd/csrc/blockgen.h"
typedef uint8_t u8; typedef uint32_t u32; typedef uint64_t u64;
static u32 rd32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static u64 rd64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }
static u32 zhash(const u8 *p, unsigned h, unsigned mls) {
    switch (mls) {
    case 5: return (u32)(((rd64(p) << 24) * 889523592379ull) >> (64 - h));
    case 6: return (u32)(((rd64(p) << 16) * 227718039650203ull) >> (64 - h));
    case 7: return (u32)(((rd64(p) << 8) * 58295818150454627ull) >> (64 - h));
    default: return (rd32(p) * 2654435761u) >> (32 - h);
    }
}
static size_t zcount(const u8 *a, const u8 *b, const u8 *aend) { const u8 *a0 = a; while (a < aend && *a == *b) { a++; b++; } return (size_t)(a - a0); }
struct Out { std::vector<u32> seq; u32 rep[2]; };
// fast parse of [bs, be) from table T (indices pos+1) and rep; FR[h] = first
// position whose read of bucket h returned an input (pre-block) value
static void fast_block(u32 *T, unsigned hlog, unsigned mls, unsigned wlog, const u8 *base, size_t bs, size_t be,
                       u32 rep[2], Out &o, std::vector<u32> &FR) {
    const u64 maxDist = 1ull << wlog;
    const u8 *const istart = base + bs, *const iend = base + be;
    const size_t prefixPos = be > maxDist ? (size_t)(be - maxDist) : 0;
    const u32 prefixIdx = (u32)prefixPos + 1;
    const u8 *const prefixStart = base + prefixPos, *const ilimit = iend - 8;
    const u8 *ip0 = istart, *ip1, *anchor = istart;
    u32 offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;
    std::fill(FR.begin(), FR.end(), 0xFFFFFFFFu);
    auto rdT = [&](u32 h, size_t pos) { const u32 v = T[h]; if (v <= bs + 1 && FR[h] == 0xFFFFFFFFu) FR[h] = (u32)pos; return v; };
    // (a value <= bs + 1 cannot be this block's own write: own writes are >= bs + 1... bs + 1 itself is pos bs)
    ip0 += (ip0 == prefixStart);
    ip1 = ip0 + 1;
    { const size_t cur = (size_t)(ip0 - base); const u32 maxRep = (u32)(cur > maxDist ? maxDist : cur);
      if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
      if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0; }
    o.seq.clear();
    while (ip1 < ilimit) {
        size_t mLength; const u8 *ip2 = ip0 + 2;
        const u32 h0 = zhash(ip0, hlog, mls), h1 = zhash(ip1, hlog, mls);
        const u32 val0 = rd32(ip0), val1 = rd32(ip1);
        const u32 current0 = (u32)(ip0 - base) + 1, current1 = (u32)(ip1 - base) + 1;
        const u32 mi0 = rdT(h0, ip0 - base), mi1 = rdT(h1, ip1 - base);
        const u8 *repMatch = ip2 - offset_1; const u8 *match0 = base + mi0 - 1, *match1 = base + mi1 - 1;
        u32 offcode;
        T[h0] = current0; T[h1] = current1;
        if ((offset_1 > 0) && rd32(repMatch) == rd32(ip2)) {
            mLength = (ip2[-1] == repMatch[-1]) ? 1 : 0; ip0 = ip2 - mLength; match0 = repMatch - mLength; mLength += 4; offcode = 0; goto match;
        }
        if (mi0 > prefixIdx && rd32(match0) == val0) goto offset;
        if (mi1 > prefixIdx && rd32(match1) == val1) { ip0 = ip1; match0 = match1; goto offset; }
        { const size_t step = ((size_t)(ip0 - anchor) >> 7) + 2; ip0 += step; ip1 += step; continue; }
    offset:
        offset_2 = offset_1; offset_1 = (u32)(ip0 - match0); offcode = offset_1 + 2; mLength = 4;
        while (ip0 > anchor && match0 > prefixStart && ip0[-1] == match0[-1]) { ip0--; match0--; mLength++; }
    match:
        mLength += zcount(ip0 + mLength, match0 + mLength, iend);
        o.seq.push_back((u32)(ip0 - anchor)); o.seq.push_back(offcode); o.seq.push_back((u32)mLength);
        ip0 += mLength; anchor = ip0;
        if (ip0 <= ilimit) {
            T[zhash(base + current0 - 1 + 2, hlog, mls)] = current0 + 2;
            T[zhash(ip0 - 2, hlog, mls)] = (u32)(ip0 - 2 - base) + 1;
            if (offset_2 > 0) {
                while (ip0 <= ilimit && rd32(ip0) == rd32(ip0 - offset_2)) {
                    const size_t rLength = zcount(ip0 + 4, ip0 + 4 - offset_2, iend) + 4;
                    const u32 t = offset_2; offset_2 = offset_1; offset_1 = t;
                    T[zhash(ip0, hlog, mls)] = (u32)(ip0 - base) + 1; ip0 += rLength;
                    o.seq.push_back(0); o.seq.push_back(0); o.seq.push_back((u32)rLength);
                    anchor = ip0;
                }
            }
        }
        ip1 = ip0 + 1;
    }
    o.rep[0] = offset_1 ? offset_1 : offsetSaved; o.rep[1] = offset_2 ? offset_2 : offsetSaved;
}

struct St { u64 ip0, anchor; u32 off1, off2, saved; };
// the serial loop's iterations whose ip0 starts in [ss, se) of block [bs, be);
// st in/out (first segment of a block: the block start state from rep)
static void fast_seg(u32 *T, unsigned hlog, unsigned mls, unsigned wlog, const u8 *base, size_t bs, size_t be,
                     size_t ss, size_t se, bool first, u32 rep[2], St &st, std::vector<u32> &seq) {
    const u64 maxDist = 1ull << wlog;
    const u8 *const iend = base + be;
    const size_t prefixPos = be > maxDist ? (size_t)(be - maxDist) : 0;
    const u32 prefixIdx = (u32)prefixPos + 1;
    const u8 *const prefixStart = base + prefixPos, *const ilimit = iend - 8;
    const u8 *ip0, *ip1, *anchor;
    u32 offset_1, offset_2, offsetSaved;
    if (first) {
        ip0 = base + bs; anchor = ip0; offset_1 = rep[0]; offset_2 = rep[1]; offsetSaved = 0;
        ip0 += (ip0 == prefixStart);
        const size_t cur = (size_t)(ip0 - base); const u32 maxRep = (u32)(cur > maxDist ? maxDist : cur);
        if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
        if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0;
    } else {
        ip0 = base + st.ip0; anchor = base + st.anchor; offset_1 = st.off1; offset_2 = st.off2; offsetSaved = st.saved;
    }
    ip1 = ip0 + 1;
    seq.clear();
    while (ip1 < ilimit && (size_t)(ip0 - base) < se) {
        size_t mLength; const u8 *ip2 = ip0 + 2;
        const u32 h0 = zhash(ip0, hlog, mls), h1 = zhash(ip1, hlog, mls);
        const u32 val0 = rd32(ip0), val1 = rd32(ip1);
        const u32 current0 = (u32)(ip0 - base) + 1, current1 = (u32)(ip1 - base) + 1;
        const u32 mi0 = T[h0], mi1 = T[h1];
        const u8 *repMatch = ip2 - offset_1; const u8 *match0 = base + mi0 - 1, *match1 = base + mi1 - 1;
        u32 offcode;
        T[h0] = current0; T[h1] = current1;
        if ((offset_1 > 0) && rd32(repMatch) == rd32(ip2)) {
            mLength = (ip2[-1] == repMatch[-1]) ? 1 : 0; ip0 = ip2 - mLength; match0 = repMatch - mLength; mLength += 4; offcode = 0; goto match;
        }
        if (mi0 > prefixIdx && rd32(match0) == val0) goto offset;
        if (mi1 > prefixIdx && rd32(match1) == val1) { ip0 = ip1; match0 = match1; goto offset; }
        { const size_t step = ((size_t)(ip0 - anchor) >> 7) + 2; ip0 += step; ip1 += step; continue; }
    offset:
        offset_2 = offset_1; offset_1 = (u32)(ip0 - match0); offcode = offset_1 + 2; mLength = 4;
        while (ip0 > anchor && match0 > prefixStart && ip0[-1] == match0[-1]) { ip0--; match0--; mLength++; }
    match:
        mLength += zcount(ip0 + mLength, match0 + mLength, iend);
        seq.push_back((u32)(ip0 - anchor)); seq.push_back(offcode); seq.push_back((u32)mLength);
        ip0 += mLength; anchor = ip0;
        if (ip0 <= ilimit) {
            T[zhash(base + current0 - 1 + 2, hlog, mls)] = current0 + 2;
            T[zhash(ip0 - 2, hlog, mls)] = (u32)(ip0 - 2 - base) + 1;
            if (offset_2 > 0) {
                while (ip0 <= ilimit && rd32(ip0) == rd32(ip0 - offset_2)) {
                    const size_t rLength = zcount(ip0 + 4, ip0 + 4 - offset_2, iend) + 4;
                    const u32 t = offset_2; offset_2 = offset_1; offset_1 = t;
                    T[zhash(ip0, hlog, mls)] = (u32)(ip0 - base) + 1; ip0 += rLength;
                    seq.push_back(0); seq.push_back(0); seq.push_back((u32)rLength);
                    anchor = ip0;
                }
            }
        }
        ip1 = ip0 + 1;
    }
    st.ip0 = (u64)(ip0 - base); st.anchor = (u64)(anchor - base); st.off1 = offset_1; st.off2 = offset_2; st.saved = offsetSaved;
}
static int seg_sim(const u8 *src, int64_t n, size_t SEG, const std::vector<Out> &ser) {
    const unsigned wlog = 19, hlog = 14, mls = 7;
    const size_t BLK = 128 << 10, tsz = 1u << hlog, per = BLK / SEG;
    const int nb = (int)((n + BLK - 1) / BLK);
    const int ns = nb * (int)per;
    std::vector<std::vector<u32>> I(ns, std::vector<u32>(tsz, 0)), W(ns, std::vector<u32>(tsz, 0)), seq(ns);
    std::vector<St> sin(ns), sout(ns);
    std::vector<u32> rin0(nb, 1), rin1(nb, 4);
    for (auto &x : sin) x = St{0, 0, 0, 0, 0};
    std::vector<char> chg(ns, 1);
    int r = 0;
    for (; r <= ns + 1; r++) {
        int nchg = 0;
        for (int s = 0; s < ns; s++) {
            if (!chg[s]) continue;
            nchg++;
            const int k = s / (int)per;
            const size_t bs = k * BLK, be = std::min<size_t>(n, bs + BLK), ss = bs + (s % per) * SEG, se = std::min(be, ss + SEG);
            std::vector<u32> T(I[s]);
            const u32 prefixIdx = (u32)(be > (1u << wlog) ? be - (1u << wlog) : 0) + 1;
            for (auto &v : T) v = std::max(v, prefixIdx);
            u32 rep[2] = {rin0[k], rin1[k]};
            St st = sin[s];
            fast_seg(T.data(), hlog, mls, wlog, src, bs, be, ss, se, s % per == 0, rep, st, seq[s]);
            sout[s] = st;
            for (size_t h = 0; h < tsz; h++) W[s][h] = T[h] > ss ? T[h] : 0;
        }
        // merge
        int any = 0;
        std::vector<u32> run(tsz, 0);
        u32 r0 = 1, r1 = 4;
        for (int s = 0; s < ns; s++) {
            const int k = s / (int)per;
            bool c = false;
            if (s % per == 0) {
                c |= rin0[k] != r0 || rin1[k] != r1;
                rin0[k] = r0; rin1[k] = r1;
            } else {
                const St &p = sout[s - 1];
                c |= memcmp(&sin[s], &p, sizeof(St)) != 0;
                sin[s] = p;
            }
            for (size_t h = 0; h < tsz; h++) {
                if (I[s][h] != run[h]) { c = true; I[s][h] = run[h]; }
                run[h] = std::max(run[h], W[s][h]);
            }
            if (s % per == per - 1) {  // block end: rep out
                const St &q = sout[s];
                r0 = q.off1 ? q.off1 : q.saved; r1 = q.off2 ? q.off2 : q.saved;
            }
            chg[s] = c; any |= c;
        }
        printf("  seg %zu KiB round %d: %d segments parsed\n", SEG >> 10, r, nchg);
        if (!any) break;
    }
    // compare with serial: concatenated segment sequences per block
    int same = 1;
    for (int k = 0; k < nb; k++) {
        std::vector<u32> cat;
        for (size_t q = 0; q < per; q++) cat.insert(cat.end(), seq[k * per + q].begin(), seq[k * per + q].end());
        same &= cat == ser[k].seq;
    }
    printf("  seg %zu KiB: settled after round %d (%d rounds), equals serial %d, wall %.2f block parses\n", SEG >> 10, r, r + 1, same, (r + 1) * (double)SEG / BLK);
    return r + 1;
}
int main(int argc, char **argv) {
    const char cls = argc > 1 ? argv[1][0] : 'T';
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 5;
    const int64_t n = argc > 3 ? strtoll(argv[3], 0, 10) : (4 << 20);
    std::vector<u8> vocab(4096 * 16), src(n + 64, 0);
    jfs_build_vocab(vocab.data());
    int64_t w = 0;
    auto emit = [&](uint8_t b) { if (w < n) src[w++] = b; };
    jfs_gen_stream(vocab.data(), cls, seed, n, emit);
    const unsigned wlog = 19, hlog = 14, mls = 7;  // > 256 KiB tier
    const size_t BLK = 128 << 10, tsz = 1u << hlog;
    const int nb = (int)((n + BLK - 1) / BLK);
    // serial reference
    std::vector<Out> ser(nb);
    { std::vector<u32> T(tsz, 0), FR(tsz); u32 rep[2] = {1, 4};
      for (int k = 0; k < nb; k++) { const size_t bs = k * BLK, be = std::min<size_t>(n, bs + BLK);
        fast_block(T.data(), hlog, mls, wlog, src.data(), bs, be, rep, ser[k], FR); rep[0] = ser[k].rep[0]; rep[1] = ser[k].rep[1]; } }
    // speculative rounds
    std::vector<std::vector<u32>> I(nb, std::vector<u32>(tsz, 0)), W(nb, std::vector<u32>(tsz, 0)), FR(nb, std::vector<u32>(tsz));
    std::vector<u32> rin0(nb, 1), rin1(nb, 4);
    std::vector<Out> out(nb);
    std::vector<char> chg(nb, 1);
    std::vector<u32> div(nb, 0);
    double work = 0, wall = 0;
    for (int r = 0; r <= nb + 1; r++) {
        int nchg = 0; double maxf = 0, sumf = 0;
        for (int k = 0; k < nb; k++) {
            if (!chg[k]) continue;
            const size_t bs = k * BLK, be = std::min<size_t>(n, bs + BLK);
            const double f = (double)(be - std::min<size_t>(std::max<size_t>(div[k], bs), be)) / (double)(be - bs);
            nchg++; maxf = std::max(maxf, f); sumf += f;
            std::vector<u32> T(I[k]);
            const u32 prefixIdx = (u32)(be > (1u << wlog) ? be - (1u << wlog) : 0) + 1;
            for (auto &v : T) v = std::max(v, prefixIdx);
            u32 rep[2] = {rin0[k], rin1[k]};
            fast_block(T.data(), hlog, mls, wlog, src.data(), bs, be, rep, out[k], FR[k]);
            for (size_t h = 0; h < tsz; h++) W[k][h] = T[h] > bs ? T[h] : 0;
        }
        work += sumf; wall += maxf;
        printf("round %d: %2d blocks parsed, re-parse fraction if resumed: max %.3f mean %.3f\n", r, nchg, maxf, nchg ? sumf / nchg : 0.0);
        // merge
        int any = 0;
        u32 r0 = 1, r1 = 4;
        std::vector<u32> run(tsz, 0);
        for (int k = 0; k < nb; k++) {
            const size_t bs = k * BLK;
            bool rc = rin0[k] != r0 || rin1[k] != r1;
            u32 d = rc ? (u32)bs : 0xFFFFFFFFu;
            bool ic = false;
            for (size_t h = 0; h < tsz; h++) {
                if (I[k][h] != run[h]) { ic = true; I[k][h] = run[h]; d = std::min(d, FR[k][h]); }
                run[h] = std::max(run[h], W[k][h]);
            }
            chg[k] = rc || ic; div[k] = d; any |= chg[k];
            rin0[k] = r0; rin1[k] = r1;
            r0 = out[k].rep[0]; r1 = out[k].rep[1];
        }
        if (!any) { printf("settled after round %d\n", r); break; }
    }
    int same = 1;
    for (int k = 0; k < nb; k++) same &= out[k].seq == ser[k].seq;
    printf("equals serial: %d; block-parse units: full %.0f rounds x %d blocks; resumed wall %.2f block parses (vs rounds), work %.2f\n", same, 0.0, nb, wall, work);
    for (size_t S : {65536ul, 32768ul, 16384ul, 8192ul}) seg_sim(src.data(), n, S, ser);
    return 0;
}
