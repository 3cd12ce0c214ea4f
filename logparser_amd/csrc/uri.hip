// gfx950 URI kernels of the logparser_amd engine (HttpUriDissector,
// QueryStringFieldDissector): k_uri_lines, its direct path k_uri_overflow,
// and the derived (type-remapped) stages k_derived_lines.  They run after
// the parse kernels, one wave per 64 lines of the batch's line index.
#include "kernels_common.h"

namespace lp {

namespace {

// ------------------------------------------------------------------ URIs
// The URI and query-string stages of a wave's 64 lines (HttpUriDissector,
// QueryStringFieldDissector), after k_parse_lines wrote the lines' status and
// spans.  Each lane's URI sources (request URI, referer, ...) are gathered
// from the input into a compact LDS buffer (only the URI bytes: a few KiB per
// wave, so many waves share a CU and hide the arena atomics and the query
// passes' latencies), with their one-plane UEV mask; then phase 2 per lane,
// a wave-aggregated arena allocation, and the query pieces spread over the
// lanes.  A wave whose URI bytes do not fit runs on the direct (HBM) path.
// compact URI bytes per wave: with its mask plane within the LDS share of a
// CU running 16 waves (config 2: 7.3 KiB per wave on average, 8.3 KiB at the
// 99th percentile; a wave needing more runs on the direct path)
constexpr uint32_t URI_CAP = 8512;
// query pieces per lane per round of the piece pass; gather rounds per batch
// (experiment builds override them: make exp XFLAGS=-DLP_URI_QR=...)
#ifndef LP_URI_QR
#define LP_URI_QR 4
#endif
#ifndef LP_URI_GR
#define LP_URI_GR 9
#endif

// Per lane: the line's URI sources.  sp[u] = a | b << 16 (line-relative, 0 =
// none), cs[u] = the compact buffer offset of line byte a.  NU: the URI
// stages this kernel instance handles (>= P.n_uri; most programs have at
// most two, whose per-lane arrays then take two registers each)
template <int NU>
struct UriLane {
    bool ok;
    int fmt;
    uint64_t ls;  // line start in the input
    RegArr<NU> sp, cs, usep;
};

template <int NU>
__device__ __forceinline__ UriLane<NU> uri_lane(const Program& P, const Columns& C, int64_t li, bool active) {
    UriLane<NU> U;
    U.sp.fill(0);
    U.cs.fill(0);
    U.usep.fill(0);
    U.ok = false;
    U.fmt = 0;
    U.ls = 0;
    if (!active) return U;
    // every column read issued before the status is known (one round trip;
    // the values of a line that is not OK are not used)
    const uint8_t st = C.status[li];
    const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[li] : 0;
    U.ls = C.line_off[li];
    const uint32_t tf = C.tok_flags[li];
    uint32_t raw[NU], kind[NU];
    for (int u = 0; u < NU; ++u) {
        raw[u] = 0;
        kind[u] = FL_FULL;
        if (u >= P.n_uri || P.uri[u].src_q >= 0) continue;
        if (P.uri[u].src_tok >= 0) {
            raw[u] = C.tok_span[P.uri[u].src_tok][li];
            kind[u] = (tf >> P.uri[u].src_tok) & 1u ? FL_NONE : FL_FULL;  // "-" -> null
        } else {
            raw[u] = C.fl_uri[P.uri[u].src_fl][li];
            kind[u] = C.fl_kind[P.uri[u].src_fl][li];
        }
    }
    U.ok = st == ST_OK;
    U.fmt = U.ok ? fmt : 0;
    if (U.ok)
        for (int u = 0; u < P.n_uri && u < NU; ++u) {
            // uri_source_cols (lp_device.h) on the values read above
            const int a = (int)(raw[u] & 0xFFFF), b = (int)(raw[u] >> 16);
            if (P.uri[u].fmt == U.fmt && P.uri[u].src_q < 0 && kind[u] != FL_NONE && b > a) U.sp.set(u, mkspan(a, b));
        }
    return U;
}


// The fast walk of URI stage u (lp_device.h uri_walk_fast) for all lines of
// the wave at once.  A line's event bytes (its UEV bits in [a, b), usep of
// them) are numbered line after line; each round, every lane takes one event
// of the wave: its byte, its class, and from ballots over its line's earlier
// events in the round plus the line's carried state (the owner lane's
// registers) what the sequential walk would know there -- whether an
// earlier event stopped the walk, the first '&' / '?' (fa), the previous
// query-piece boundary, the last '%' / '+'.  A boundary event that ends a
// non-empty piece writes its table slot; at the end of each round every
// owner lane folds its events of the round into its state.  The result per
// lane (part: the lane's line takes part) is exactly the sequential walk's
// state: resume, fa, first_pct, rewr bit 1, the query table (slots, count,
// s, lp).  L: the lane's line view (compact buffer with its UEV plane);
// A.p / A.used: the line's region and where its table starts.
// SLOT: u differs between lanes (the k-th URI stage of each lane's own
// LogFormat, -1 none): an event takes its owner line's table flag.
template <bool SLOT, typename CL>
__device__ __forceinline__ void uri_walk_coop(const Program& P, int u, const CL& L, bool part, int a, int b,
                                              uint32_t usep, const Arena& A, UriWalk& Wk) {
    const int lane = lane_id();
    const bool table = u >= 0 && P.uri[u].want_query && P.uri[u].query_stage >= 0;  // uniform unless SLOT
    const uint32_t cnt = part ? usep : 0u;
    uint32_t x = cnt;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t eb = x - cnt, E = __shfl(x, 63);
    const uint32_t tab = (A.used + 15) & ~15u;
    const unsigned long long reg = (unsigned long long)(uintptr_t)A.p;
    // the owner's state (this lane's line)
    int resume = -1, fa = -1, fpct = -1, lastB = -1, lastPP = -1;
    uint32_t count = 0;
    bool rw = false;
    for (uint32_t g0 = 0; g0 < E; g0 += PW) {
        const uint32_t g = g0 + (uint32_t)lane;
        const bool valid = g < E;
        int ow = 0;  // last lane whose first event is <= g
        for (int st = 32; st; st >>= 1)
            if (__shfl((int)eb, ow + st) <= (int)g) ow += st;
        const uint32_t ebo = (uint32_t)__shfl((int)eb, ow);
        const uint32_t oo = (uint32_t)__shfl((int)L.o, ow);
        const int oa = __shfl(a, ow), ob = __shfl(b, ow);
        // the event: the (g - ebo)-th UEV bit of the owner's [oa, ob)
        uint32_t Aq = 0;
        if (valid) {
            const uint32_t A0 = oo + (uint32_t)oa, A1 = oo + (uint32_t)ob, WL = (A1 - 1) >> 6;
            uint32_t W = A0 >> 6, k = g - ebo;
            uint64_t m = L.mask(MC_UEV, W) & (~0ull << (A0 & 63));
            for (;;) {
                if (W == WL) m &= ~0ull >> (63 - ((A1 - 1) & 63));
                const uint32_t c = (uint32_t)__popcll(m);
                if (k < c || W >= WL) break;  // (the count came from the same plane: k < c by WL)
                k -= c;
                ++W;
                m = L.mask(MC_UEV, W);
            }
            Aq = (W << 6) + select64(m, k);
        }
        const int q = (int)(Aq - oo);
        CL Lo = L;
        Lo.o = oo;
        Lo.n = ob;
        const uint32_t w = valid ? load_u32_at(Lo, q) : 0u;
        const uint32_t c = w & 0xFFu;
        const bool pct = c == '%';
        const bool bad_pct = pct && (q + 2 >= ob || !is_hex((w >> 8) & 0xFFu) || !is_hex((w >> 16) & 0xFFu));
        const bool stop = valid && (c == '#' || c == ';' || c >= 0x80 || bad_pct);
        const bool aq = c == '&' || c == '?';
        // the owner's state before this round
        const int cres = __shfl(resume, ow), cfa = __shfl(fa, ow), clB = __shfl(lastB, ow), clPP = __shfl(lastPP, ow);
        const uint32_t ccount = (uint32_t)__shfl((int)count, ow);
        // my line's earlier events in this round: lanes [seg0, lane)
        const int s0 = (int)ebo - (int)g0;
        const uint64_t below = (1ull << lane) - 1ull;
        const uint64_t seg_lt = valid ? below & (~0ull << (s0 > 0 ? s0 : 0)) : 0ull;
        const uint64_t Bstop = __ballot(stop);
        const bool live = valid && !stop && cres < 0 && !(Bstop & seg_lt);  // the fast walk takes this event
        const uint64_t Baq = __ballot(live && aq);
        const uint64_t mfa = Baq & seg_lt;
        const int qfa = __shfl(q, mfa ? lsb64(mfa) : lane);
        const int fa_j = cfa >= 0 ? cfa : (mfa ? qfa : -1);  // the first '&' / '?' before me
        const bool pp = live && ((pct && !bad_pct) || c == '+');
        const bool otable = SLOT ? __shfl((int)table, ow) != 0 : table;  // the owner line's stage has a table
        const bool isB = otable && live && aq && fa_j >= 0;  // a piece boundary after fa
        const uint64_t BB = __ballot(isB), BPP = __ballot(pp);
        const uint64_t mB = BB & seg_lt, mP = BPP & seg_lt;
        const int qpb = __shfl(q, mB ? msb64(mB) : lane), qpp = __shfl(q, mP ? msb64(mP) : lane);
        const bool first_piece = !mB && clB < 0;  // the previous boundary is fa
        const int pb = mB ? qpb : (clB >= 0 ? clB : fa_j);
        const int lpp = mP ? qpp : clPP;  // the last '%' / '+' before me
        const int lp = first_piece ? lpp : (lpp > pb ? lpp : -1);
        const bool emit = isB && q > pb + 1;
        const uint64_t BE = __ballot(emit);
        const bool rwj = live && fa_j >= 0 && ((aq && c == '?') || (!aq && !pct && uri_needs_encode(c)));
        const uint64_t BR = __ballot(rwj);
        const unsigned long long oreg = __shfl(reg, ow);
        const uint32_t otab = (uint32_t)__shfl((int)tab, ow);
        if (emit) {
            const uint32_t idx = ccount + (uint32_t)__popcll(BE & seg_lt);
            const uint64_t t0 = (uint64_t)(uint32_t)(pb + 1) | ((uint64_t)(uint32_t)q << 16) | ((uint64_t)(uint32_t)(lp + 1) << 48);
            *reinterpret_cast<LP_G u32x4*>(reinterpret_cast<LP_G uint8_t*>(oreg) + otab + 16 * idx) =
                u32x4{(uint32_t)t0, (uint32_t)(t0 >> 32), 0u, 0u};
        }
        // owners fold their events of this round into their state
        const int so = (int)eb - (int)g0, eo = (int)(eb + cnt) - (int)g0;
        const int so_c = so < 0 ? 0 : so > PW ? PW : so, eo_c = eo < 0 ? 0 : eo > PW ? PW : eo;
        const uint64_t segm = so_c < eo_c ? ((eo_c == PW ? ~0ull : (1ull << eo_c) - 1ull) & (~0ull << so_c)) : 0ull;
        const uint64_t ms = Bstop & segm, mf = Baq & segm, mpct = __ballot(live && pct) & segm, mb = BB & segm,
                       mpp = BPP & segm;
        const int q_s = __shfl(q, ms ? lsb64(ms) : lane), q_f = __shfl(q, mf ? lsb64(mf) : lane);
        const int q_p = __shfl(q, mpct ? lsb64(mpct) : lane), q_b = __shfl(q, mb ? msb64(mb) : lane);
        const int q_pp = __shfl(q, mpp ? msb64(mpp) : lane);
        if (resume < 0 && ms) resume = q_s;
        if (fa < 0 && mf) fa = q_f;
        if (fpct < 0 && mpct) fpct = q_p;
        if (mb) lastB = q_b;
        if (mpp) lastPP = q_pp;
        count += (uint32_t)__popcll(BE & segm);
        rw = rw || (BR & segm) != 0;
    }
    if (!part) return;
    Wk.resume = resume;
    Wk.fa = fa;
    Wk.first_pct = fpct;
    Wk.rewr = rw ? 2u : 0u;
    QueryTable& T = Wk.T;
    if (table && fa >= 0) {
        T.on = T.set = true;
        T.maxp = usep + 1;
        T.tab = tab;
        T.reg = tab + 16 * T.maxp;
        T.s = (lastB >= 0 ? lastB : fa) + 1;
        T.count = count;
        T.lp = lastB >= 0 ? (lastPP > lastB ? lastPP : -1) : lastPP;
    } else {
        T.lp = lastPP;
    }
}

// Phase 2, the arena allocation and the query pieces of one wave; lu(u) is
// the lane's line view of URI stage u (valid for every lane, empty stages
// included: the query pass reads other lanes' views).
// SLOT (several LogFormats): pass k runs, on every lane, the k-th URI stage of
// the lane's own LogFormat (URI stages by slot: the lanes of all formats
// walk together instead of each format's stages under a partial mask).
template <int NU, int NQ, bool COOP, bool SLOT, typename LU, typename LL>
__device__ __forceinline__ void uri_wave(const Program& P, const Columns& C, UriLane<NU>& U, LU&& lu, LL&& ll,
                                         bool active, int64_t li, int64_t wave, WaveCounts& WC) {
    const int lane = lane_id();
    const int nq = P.n_query < NQ ? P.n_query : NQ;
    uint32_t need = 0;
    if (U.ok)
        for (int u = 0; u < P.n_uri && u < NU; ++u) {
            const uint32_t s = U.sp.get(u);
            if (!s) continue;
            uint32_t ev;
            need += uri_need(P, u, lu(u), (int)(s & 0xFFFF), (int)(s >> 16), ev);
            U.usep.set(u, ev);
        }
    // upstream list stages (UpstreamListDissector): their item tables follow
    // the URI stages' in the line's region (and the name / value pieces of
    // cookie headers and raw query strings); ll(lend) views the list / pair
    // token bytes (gathered into LDS beside the URI bytes, or in HBM)
    int lend = 0;
    if (U.ok) {
        for (int j = 0; j < P.n_list; ++j)
            if (P.list[j].fmt == U.fmt) lend = max(lend, (int)(C.tok_span[P.list[j].tok][li] >> 16));
        for (int j = 0; j < P.n_pair; ++j)
            if (P.pair[j].fmt == U.fmt) lend = max(lend, (int)(C.tok_span[P.pair[j].tok][li] >> 16));
    }
    if (lend) ll(lend, [&](const auto& LH) { need += list_need(P, U.fmt, LH, C, li) + pair_need(P, U.fmt, LH, C, li); });
    need = (need + 15) & ~15u;
    // wave-aggregated arena allocation from the wave's shard
    uint32_t x = need;
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, 63);
    const int shard = (int)(wave % ARENA_SHARDS);
    unsigned long long wbase = 0;
    // regions start 16-byte aligned (their query tables take 16-byte slot
    // stores; spills keep the bump pointer only 4-byte aligned)
    if (lane == 63 && total) wbase = atomicAdd(&C.meta->shard_top[16 * shard], (unsigned long long)total + 12ull);
    wbase = (__shfl(wbase, 63) + 15) & ~15ull;
    const bool fits = wbase + total <= C.shard_cap;
    LP_PROF(26);
    uint32_t written = 0;
    unsigned long long my_region = 0;
    UriOutT<NQ> o;
    o.qlist.fill(0);
    o.qpend.fill(0);
    o.status = U.ok ? ST_OK : ST_BAD;
    Arena A{C.arena, 0, 0};
    bool live = false;  // the line's region is allocated: phase 2 runs
    if (U.ok) {
        if (!fits && need) {
            // the shard is full: the batch is re-run with a larger arena
            o.status = ST_FALLBACK;
            atomicAdd(&C.meta->arena_ovf, 1ull);
        } else {
            const unsigned long long mine = (unsigned long long)shard * C.shard_cap + wbase + x - need;
            my_region = mine;
            C.arena_base[li] = mine;  // also for an empty region: spills are region-relative
            A = Arena{C.arena + mine, 0, need};
            A.top = &C.meta->shard_top[16 * shard];  // spills come from the same shard
            A.base = wbase + x - need;
            A.limit = C.shard_cap;
            live = true;
        }
    }
    // phase 2 (lp_device.h phase2), stage by stage for the whole wave: the
    // compact path walks the stages' event bytes cooperatively
    const int nu = P.n_uri < NU ? P.n_uri : NU;
    for (int sl = 0; sl < nu; ++sl) {
        int u = sl;  // this lane's stage of the pass
        if constexpr (SLOT) {
            u = -1;
            for (int v = 0, c = 0; v < nu; ++v)
                if (P.uri[v].fmt == U.fmt) {
                    if (c == sl) u = v;
                    ++c;
                }
            if (!__any(u >= 0)) break;  // no lane's LogFormat has a sl-th stage
        }
        const bool fmt_ok = live && o.status == ST_OK && u >= 0 && P.uri[u].fmt == U.fmt;
        const uint32_t sp = U.sp.get(u);
        const int a = (int)(sp & 0xFFFF), b = (int)(sp >> 16);
        const bool part = fmt_ok && b > a;
        if (fmt_ok && !part) {
            C.u_flags[u][li] = 0;
            if (P.uri[u].query_stage >= 0) { C.q_count[P.uri[u].query_stage][li] = 0; C.q_params[P.uri[u].query_stage][li] = 0; }
        }
        LP_PROF(10 + 2 * sl);
        UriWalk Wk;
        if constexpr (COOP) {
            LP_PROF(50 + 4 * sl);
            uri_walk_coop<SLOT>(P, u, lu(u), part, a, b, U.usep.get(u), A, Wk);
            LP_PROF(51 + 4 * sl);
        } else if (part) {
            uri_walk_fast(P, u, lu(u), a, b, U.usep.get(u), A, Wk);
        }
        if (part) {
            const int st = uri_stage_rest(P, u, lu(u), a, b, U.usep.get(u), A, C, li, o, Wk);
            if (st != ST_OK) o.status = st;
        }
        LP_PROF(11 + 2 * sl);
    }
    if (live && lend && o.status == ST_OK) {
        bool filled = true;
        ll(lend, [&](const auto& LH) { filled = list_fill(P, U.fmt, LH, A, C, li) && pair_fill(P, U.fmt, LH, A, C, li); });
        if (!filled) o.status = ST_FALLBACK;
    }
    if (live) {
        if (A.ovf) {
            o.status = ST_FALLBACK;
            atomicAdd(&C.meta->arena_ovf, 1ull);
        }
        written = A.used - A.slack + A.extra;
    }
    LP_PROF(21);
    // QueryStringFieldDissector pieces of all lines of the wave, spread evenly
    // over the lanes (a line's pieces vary from 0 to dozens; one lane per line
    // would leave most lanes idle while the longest query finishes): the
    // pieces of every query stage in one numbering (a lane's stage-0 pieces,
    // then its stage-1 pieces, ...), QR blocks of 64 pieces per round: their
    // table slots loaded together, then query_prep, ONE spill allocation for
    // the round, query_finish.  Most waves need one round for all stages.
    if (nq > 0) {
        constexpr int QR = LP_URI_QR;
        __syncthreads();  // the table slots written in phase 2 are visible to every lane
        const bool has = U.ok && o.status == ST_OK && need != 0;
        const unsigned long long my_ab = has ? my_region : 0ull;
        uint64_t piece_ovf = 0;  // lanes whose line lost a piece for want of arena
        uint32_t np = 0;
        for (int qs = 0; qs < nq; ++qs) np += has ? o.qpend.get(qs) : 0u;
        uint32_t incl = np;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t base = incl - np, tot = __shfl(incl, 63);
        // piece j of lane ow: its query stage and its slot in ow's region;
        // OL = ow's line view of that stage (every lane takes part in the shuffles)
        auto piece = [&](int ow, uint32_t j, int& pq, uint32_t& soff) {
            uint32_t cum = 0;
            pq = 0;
            soff = 0;
            for (int qs = 0; qs < nq; ++qs) {
                const uint32_t c = (uint32_t)__shfl((int)(has ? o.qpend.get(qs) : 0u), ow);
                const uint32_t l = (uint32_t)__shfl((int)o.qlist.get(qs), ow);
                if (j >= cum && j < cum + c) {
                    pq = qs;
                    soff = l + 16 * (j - cum);
                }
                cum += c;
            }
        };
        auto owner_view = [&](int ow, int pq) {
            auto OL = owner_line(lu(P.query[0].uri), ow);
            for (int qs = 1; qs < nq; ++qs) {
                const auto V = owner_line(lu(P.query[qs].uri), ow);
                if (pq == qs) OL = V;
            }
            return OL;
        };
        for (uint32_t g0 = 0; g0 < tot; g0 += QR * PW) {
            int own[QR], pqs[QR];
            uint32_t soffs[QR];
            uint64_t t0[QR];
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                own[k] = 0;
                pqs[k] = 0;
                soffs[k] = 0;
                t0[k] = 0;
                if (g0 + (uint32_t)(k * PW) >= tot) continue;  // no piece in this block (uniform)
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                int ow = 0;  // last lane whose first pending piece index is <= g
                for (int st = 32; st; st >>= 1)
                    if (__shfl(base, ow + st) <= g) ow += st;
                own[k] = ow;
                const uint32_t ob = __shfl(base, ow);
                const unsigned long long oab = __shfl(my_ab, ow);
                piece(ow, g - ob, pqs[k], soffs[k]);
                if (g < tot) t0[k] = *reinterpret_cast<const LP_G uint64_t*>(C.arena + oab + soffs[k]);
            }
            LP_PROF(17);
            QPrep qp[QR];
            uint32_t mine = 0;
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                if (g0 + (uint32_t)(k * PW) >= tot) continue;
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                const auto OL = owner_view(own[k], pqs[k]);
                if (g < tot) qp[k] = query_prep(OL, t0[k]);
                mine += qp[k].need;
            }
            LP_PROF(18);
            // the round's spilled bytes in one allocation from the wave's
            // shard (every owner is a line of this wave)
            uint32_t x = mine;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            const uint32_t rtot = __shfl(x, 63);
            unsigned long long rbase = 0;
            if (lane == 63 && rtot) rbase = atomicAdd(&C.meta->shard_top[16 * shard], (unsigned long long)rtot);
            unsigned long long at = __shfl(rbase, 63) + x - mine;  // this lane's first piece in the shard
            LP_PROF(19);
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                if (g0 + (uint32_t)(k * PW) >= tot) continue;
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                const int ow = own[k];
                const unsigned long long oab = __shfl(my_ab, ow);
                const auto OL = owner_view(ow, pqs[k]);
                bool povf = false;
                if (g < tot) {
                    LP_G uint64_t* slot = reinterpret_cast<LP_G uint64_t*>(C.arena + oab + soffs[k]);
                    const unsigned long long rel = oab - (unsigned long long)shard * C.shard_cap;  // region in the shard
                    if (qp[k].need && (at + qp[k].need > C.shard_cap || at - rel + qp[k].need > 0x7FFFFFFFull)) {
                        slot[0] = REF_SKIP;
                        slot[1] = 0;
                        povf = true;
                        atomicAdd(&C.meta->arena_ovf, 1ull);  // the batch is re-run with a larger arena
                    } else {
                        Arena A{C.arena + oab, (uint32_t)(at - rel), (uint32_t)(at - rel + qp[k].need)};
                        written += query_finish(P, P.query[pqs[k]], OL, A, C.arena + oab, slot, qp[k]);
                    }
                    at += qp[k].need;
                }
                // a piece that did not fit: its line goes to FALLBACK (the
                // batch is re-run with a larger arena, or, when the re-runs
                // are spent, delivered with those lines FALLBACK)
                for (uint64_t m = __ballot(povf); m; m &= m - 1) piece_ovf |= 1ull << __shfl(ow, (int)__builtin_ctzll(m));
            }
        }
        if (((piece_ovf >> lane) & 1) && o.status == ST_OK) o.status = ST_FALLBACK;
    }
    LP_PROF(22);
    if (U.ok && o.status != ST_OK) C.status[li] = (uint8_t)o.status;
    for (int d = 32; d > 0; d >>= 1) written += __shfl_xor(written, d);
    const int st = !active ? -1 : U.ok ? o.status : (int)C.status[li];
    WC.act += (uint32_t)__popcll(__ballot(active));
    WC.ok += (uint32_t)__popcll(__ballot(st == ST_OK));
    WC.bad += (uint32_t)__popcll(__ballot(st == ST_BAD));
    WC.written += written;
}


// The URI stages of one wave on the compact path: its lines' URI bytes
// gathered into cbuf (CAP bytes) with their UEV plane, then uri_wave.
// Returns false, having done nothing, when the wave's bytes exceed CAP.
template <int NU, int NQ, bool SLOT, uint32_t CAP>
__device__ __forceinline__ bool uri_compact(const uint8_t* __restrict__ buf, uint64_t nbytes, const Program& P,
                                            const Columns& C, int64_t wave, int64_t n_lines, uint32_t* cbuf,
                                            uint64_t* plane, WaveCounts& WC) {
    const int lane = lane_id();
    const int64_t li = wave * PW + lane;
    const bool active = li < n_lines;
    LP_PROF(23);
    UriLane<NU> U = uri_lane<NU>(P, C, li, active);
    LP_PROF(27);
    // one region per line: the 16-byte input blocks holding all its URI
    // sources (request URI, referer, ...: close together in a line), in
    // line order; a block keeps its alignment, so the wave gathers whole
    // aligned 16-byte blocks, consecutive lanes taking consecutive blocks
    uint64_t lo = ~0ull, hi = 0;
    for (int u = 0; u < P.n_uri && u < NU; ++u) {
        const uint32_t s = U.sp.get(u);
        if (!s) continue;
        lo = min(lo, U.ls + (s & 0xFFFF));
        hi = max(hi, U.ls + (s >> 16));
    }
    const uint64_t r0 = hi ? lo & ~15ull : 0;
    const uint32_t nb1 = hi ? (uint32_t)((((hi + 15) & ~15ull) - r0) >> 4) : 0u;
    // the line's list / pair tokens (upstream lists, cookie headers, raw
    // query strings): a second region of blocks after the URI ones
    const bool lists = P.n_list > 0 || P.n_pair > 0;  // wave-uniform
    uint64_t l0 = ~0ull, l1 = 0;
    if (lists && U.ok) {
        auto add = [&](int tok) {
            const uint32_t s = C.tok_span[tok][li];
            if ((s >> 16) > (s & 0xFFFFu)) {
                l0 = min(l0, U.ls + (s & 0xFFFFu));
                l1 = max(l1, U.ls + (s >> 16));
            }
        };
        for (int j = 0; j < P.n_list; ++j)
            if (P.list[j].fmt == U.fmt) add(P.list[j].tok);
        for (int j = 0; j < P.n_pair; ++j)
            if (P.pair[j].fmt == U.fmt) add(P.pair[j].tok);
    }
    const uint64_t q0 = l1 ? l0 & ~15ull : 0;
    const uint32_t nb2 = l1 ? (uint32_t)((((l1 + 15) & ~15ull) - q0) >> 4) : 0u;
    auto blocks = [&](uint32_t n, uint32_t& first) {  // the wave's block count, this line's first block
        uint32_t x = n;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        first = x - n;
        return (uint32_t)__shfl(x, 63);
    };
    uint32_t cb;
    uint32_t tot = blocks(nb1 + nb2, cb);
    // the list / pair tokens in LDS when the wave's bytes fit with them, else
    // read from HBM (only the URI bytes decide whether the wave fits)
    bool lin = lists;
    if (lists && 16 * tot + 16 > CAP) {
        lin = false;
        tot = blocks(nb1, cb);
    }
    if (16 * tot + 16 > CAP) return false;
    WC.gathered = 16 * tot;
    for (int u = 0; u < P.n_uri && u < NU; ++u) {
        const uint32_t s = U.sp.get(u);
        if (s) U.cs.set(u, 16 * cb + (uint32_t)(U.ls + (s & 0xFFFF) - r0));
    }
    // gather: block g of the wave is block g - cb[own] of line own's region,
    // own = the last lane whose first block is <= g; every round's load in
    // flight before the first store
    constexpr int GR = LP_URI_GR;  // rounds per batch (the main kernel's CAP / 1024, rounded up)
    uint16_t* pl16 = reinterpret_cast<uint16_t*>(plane);
    for (uint32_t g0 = 0; g0 < tot; g0 += GR * PW) {
        u32x4 v[GR];
#pragma unroll
        for (int k = 0; k < GR; ++k) {
            const uint32_t g = g0 + (uint32_t)(k * PW + lane);
            int own = 0;
            for (int st = 32; st; st >>= 1)
                if (__shfl(cb, own + st) <= g) own += st;
            const uint32_t j = g - (uint32_t)__shfl(cb, own);  // block j of line own's regions
            uint64_t src = (uint64_t)__shfl((unsigned long long)r0, own) + 16ull * j;
            if (lin) {  // (every lane in the shuffles: a permute reads no value from an inactive lane)
                const uint32_t n1 = (uint32_t)__shfl(nb1, own);
                const uint64_t s1 = (uint64_t)__shfl((unsigned long long)q0, own);
                if (j >= n1) src = s1 + 16ull * (j - n1);
            }
            v[k] = u32x4{0, 0, 0, 0};
            if (g < tot) v[k] = load16(buf, nbytes, src);
        }
        LP_PROF(28);
#pragma unroll
        for (int k = 0; k < GR; ++k) {
            const uint32_t g = g0 + (uint32_t)(k * PW + lane);
            if (g >= tot) continue;
            *reinterpret_cast<u32x4*>(cbuf + 4 * g) = v[k];
            pl16[g] = (uint16_t)bcls::classify16u(v[k][0], v[k][1], v[k][2], v[k][3]);
        }
    }
    LP_PROF(24);
    // one zero block after the last (the scanners' look-ahead word) and the
    // rest of the last 64-byte mask block
    for (uint32_t g = tot + lane; g < ((tot + 1 + 3) & ~3u); g += PW) {
        *reinterpret_cast<u32x4*>(cbuf + 4 * g) = u32x4{0, 0, 0, 0};
        pl16[g] = 0;
    }
    __syncthreads();
    LP_PROF(25);
    typedef LineT<lds_bytes, lds_u64, 1> CL;
    auto lu = [&](int u) {
        const uint32_t s = U.sp.get(u);
        // line byte q lives at cbuf + cs + (q - a): origin cs - a (mod 2^32)
        return CL{(lds_bytes)cbuf, U.cs.get(u) - (s & 0xFFFFu), (int)(s >> 16), (lds_u64)plane};
    };
    // line byte q of a list / pair token at cbuf + 16 (cb + nb1) + (q - (q0 - ls)),
    // or in place in the input; ll(lend, f) runs f on the view (lin is
    // wave-uniform: LDS or global loads, never flat ones)
    const LP_G uint8_t* lsp = (const LP_G uint8_t*)buf + U.ls;
    const uint32_t lmis = (uint32_t)((uintptr_t)lsp & 3);
    const uint32_t lorig = 16 * (cb + nb1) + (uint32_t)(U.ls - q0);
    auto ll = [&](int lend, auto&& f) {
        if (lin) f(LineT<lds_bytes>{(lds_bytes)cbuf, lorig, lend});
        else f(LineT<const LP_G uint8_t*>{lsp - lmis, lmis, lend});
    };
    uri_wave<NU, NQ, true, SLOT>(P, C, U, lu, ll, active, li, wave, WC);
    return true;
}

// 16 waves per CU: the LDS share allows them, and __launch_bounds__(64, 4)
// (4 waves per SIMD) keeps the registers within 128
#ifndef LP_URI_SLOT_WPE
#define LP_URI_SLOT_WPE 4  // waves per SIMD of the several-format (SLOT) instance
#endif
template <int NU, int NQ, bool SLOT>
__global__ __launch_bounds__(PW, SLOT ? LP_URI_SLOT_WPE : 4) void k_uri_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    __shared__ __attribute__((aligned(16))) uint32_t cbuf[URI_CAP / 4 + 16];
    __shared__ uint64_t plane[URI_CAP / 64 + 1];
    WaveCounts WC;
    if (uri_compact<NU, NQ, SLOT, URI_CAP>(buf, nbytes, P, C, wave, n_lines, cbuf, plane, WC)) WC.store(C, wave);
    else if (lane_id() == 0) C.uri_ovf_list[atomicAdd(&C.meta->uri_ovf_waves, 1ull)] = (uint32_t)wave;
}

// The waves k_uri_lines queued (their URI bytes exceed its compact buffer),
// on a persistent grid: the same path with a buffer four times as large (few
// waves: their occupancy does not matter), and for a wave exceeding even
// that, the lines' bytes read from HBM directly.
constexpr uint32_t URI_CAP_OVF = 4 * URI_CAP;
template <int NU, int NQ, bool SLOT>
__global__ __launch_bounds__(PW) void k_uri_overflow(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const uint64_t nq = C.meta->uri_ovf_waves;
    __shared__ __attribute__((aligned(16))) uint32_t cbuf[URI_CAP_OVF / 4 + 16];
    __shared__ uint64_t plane[URI_CAP_OVF / 64 + 1];
    for (uint64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t wave = C.uri_ovf_list[q];
        WaveCounts WC;
        if (!uri_compact<NU, NQ, SLOT, URI_CAP_OVF>(buf, nbytes, P, C, wave, n_lines, cbuf, plane, WC)) {
            const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
            UriLane<NU> U = uri_lane<NU>(P, C, W.li, W.active);
            const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
            const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
            const LineT<const LP_G uint8_t*> L{ls - mis, mis, crlf_len_hbm(buf, W)};
            auto lu = [&](int) { return L; };
            auto ll = [&](int lend, auto&& f) { f(LineT<const LP_G uint8_t*>{ls - mis, mis, lend}); };
            uri_wave<NU, NQ, false, SLOT>(P, C, U, lu, ll, W.active, W.li, wave, WC);
        }
        __syncthreads();
        WC.store(C, wave);
    }
}

// Derived URI stages (type-remapped query parameters, lp_device.h
// derived_line), after both URI kernels: one line per lane, the sources read
// in place (the input, or the decoded value in the line's region), every
// table and rewritten part spilled from the region's shard.  Only launched
// for programs that have such stages.  Re-counts the wave's statuses.
__global__ __launch_bounds__(PW) void k_derived_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                      const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
    int st = W.active ? (int)C.status[W.li] : -1;
    if (st == ST_OK) {
        const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[W.li] : 0;
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const unsigned long long ab = C.arena_base[W.li];
        const int shard = (int)(ab / C.shard_cap);
        Arena R{C.arena + ab, 0, 0};
        R.top = &C.meta->shard_top[16 * shard];
        R.base = ab - (unsigned long long)shard * C.shard_cap;
        R.limit = C.shard_cap;
        st = derived_line(P, fmt, ls - mis, mis, crlf_len_hbm(buf, W), R, C, W.li);
        if (R.ovf) atomicAdd(&C.meta->arena_ovf, 1ull);  // the batch is re-run with a larger arena
        if (st != ST_OK) C.status[W.li] = (uint8_t)st;
    }
    const uint32_t ok = (uint32_t)__popcll(__ballot(st == ST_OK)), bad = (uint32_t)__popcll(__ballot(st == ST_BAD));
    if (lane_id() == 0) {
        LP_G uint32_t* wc = C.wave_counts + WC_WORDS * (size_t)wave;
        const uint32_t act = wc[0];
        wc[1] = ok;
        wc[2] = bad;
        wc[3] = act - ok - bad;
    }
}

}  // namespace

int launch_uri(const ParseLaunch& a, const DeviceArgs* d_args, hipStream_t s) {
    const int64_t waves = parse_waves(a.cap_lines);
    if (waves == 0 || !a.uri) return 0;
    const int64_t grid = waves < 1024 ? waves : 1024;
    // most programs have at most two URI and two query stages (the request
    // URI and the referer): an instance keeping two of each
    // several LogFormats (not a.chunked): the instance running URI stages by slot
    if (!a.chunked) {
        hipLaunchKernelGGL((k_uri_lines<MAX_URI, MAX_QUERY, true>), dim3((unsigned)waves), dim3(PW), 0, s, a.buf,
                           a.nbytes, d_args);
        hipLaunchKernelGGL((k_uri_overflow<MAX_URI, MAX_QUERY, true>), dim3((unsigned)grid), dim3(PW), 0, s, a.buf,
                           a.nbytes, d_args);
    } else if (a.n_uri <= 2 && a.n_query <= 2) {
        hipLaunchKernelGGL((k_uri_lines<2, 2, false>), dim3((unsigned)waves), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
        hipLaunchKernelGGL((k_uri_overflow<2, 2, false>), dim3((unsigned)grid), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
    } else {
        hipLaunchKernelGGL((k_uri_lines<MAX_URI, MAX_QUERY, false>), dim3((unsigned)waves), dim3(PW), 0, s, a.buf,
                           a.nbytes, d_args);
        hipLaunchKernelGGL((k_uri_overflow<MAX_URI, MAX_QUERY, false>), dim3((unsigned)grid), dim3(PW), 0, s, a.buf,
                           a.nbytes, d_args);
    }
    if (a.derived) hipLaunchKernelGGL(k_derived_lines, dim3((unsigned)waves), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#if defined(LP_PROFILE)
int prof_read_uri(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * PROF_WAVES * PROF_POINTS) == hipSuccess ? 0 : -1;
}
int prof_clear_uri() {
    static unsigned long long z[PROF_WAVES * PROF_POINTS];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace lp
