// ldpc5g_dec_split.hip — float64 flooding min-sum decoder for a FEW LARGE codeblocks: the launch
// shape of the per-codeblock drop-ins at Zc >= 64 (nr_decode_ldpc decodes one codeblock per call, so
// its latency is one codeblock's, not a batch's).  Each codeblock is spread over
// W = ceil(MB * ceil(Zc/64) / 16) workgroups of 1024 threads, one per CU (W = 18 for BG1 Zc = 384), instead of
// the batch kernel's one workgroup per codeblock.
//
// Same arithmetic in the same order as the small-codeblock kernel (ldpc5g_dec_small.h), hence
// bit-identical to py5gphy/ldpc/nr_ldpc_decode.py:51-143 with _min_sum_process :178-227:
//   phase A  a thread per check node (base row i, z): reads LQ_old of its row's edges at
//            (z + V) mod Zc, the syndrome of LQ_old's hard decisions (:107-114) from the same reads,
//            new row state (:117-123, :186-202), and its core edges' new messages r written to their
//            message slots in CSC order (column j's edges rows ascending) at row (z + V) mod Zc;
//   phase B  a thread per core column entry (j, z): LQ = LLRin + the column's messages summed rows
//            ascending (Lr.sum(axis=0), :126) — consecutive slots, all loads in flight together.
// LQ and the messages live in a global scratch (per codeblock (KC + NCE) * Zc doubles, 0.84 MB for
// BG1 Zc = 384) instead of LDS, and the two barriers per iteration are barriers over the codeblock's
// W workgroups: one monotonic counter per codeblock; every hand-off store (LQ, messages, flags) is an
// `sc1` (write-through) store, every storing wave drains (vmcnt(0)) before the workgroup barrier
// behind which one lane adds to the counter, the counter is polled with an `sc1` load and every load
// of hand-off data is an `sc1` global load (MI355X_MICROARCH.md, hand-off table first row): no L2
// write-back or L1 invalidate fence on the critical path.  A codeblock's W workgroups must be
// resident together: workgroups take their (codeblock, part) by an arrival ticket, so parts go to
// resident workgroups in order and at most one codeblock per launch waits for CUs; the launcher keeps
// B*W <= kSplitMaxWG (224 of the 256 CUs), one workgroup per CU, and chains the split launches of a
// device (in one process) one after another across streams (an event per device).  Launches of
// more codeblocks take R = 2 chunks per wave (half the workgroups per codeblock).
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>

#include "ldpc5g_dec_small.h"

namespace ldpc5g_impl {
namespace {

constexpr int kSplitThreads = 1024;
constexpr int kSplitSync = 64;   // sync words per codeblock (a 256-B line): barrier counter, flags
constexpr int kSplitMaxWG = 224;   // of the 256 CUs, one workgroup each (7/8 of a device's CUs)
// A barrier wait gives up after this many ticks of the 100 MHz real-time clock (4 s; a barrier takes
// microseconds).  The parts of a codeblock must be resident together; if some never get a CU (other
// kernels holding the device), the waiting parts abort instead of hanging the GPU: bit 31 of the
// codeblock's barrier counter (sticky: every part's poll ends on it), status 0, iters -1, the
// device's timeout count + 1 (ldpc5g_split_timeouts), and the last part out clears the sync words.
constexpr uint64_t kSplitTimeoutTicks = 400000000ull;
constexpr uint32_t kSplitAbort = 0x80000000u;
// loads in flight per chunk (phase A LQ reads, phase B message reads); 32: a row's / column's all
// at once (r05, one BG1 Zc=384 codeblock: 10 / 10 100 us per call, all 87 us)
#ifndef LDPC5G_SPLIT_CH
#define LDPC5G_SPLIT_CH 32
#endif
#ifndef LDPC5G_SPLIT_CCH
#define LDPC5G_SPLIT_CCH 32
#endif
// development instrumentation (tools/split_probe.py): workgroup 0 thread 0's real-time clock
// (100 MHz) at phase boundaries, dumped over its codeblock's decisions (codeblock 0 when workgroup 0
// takes the first ticket, as it does when dispatched first)
#ifdef LDPC5G_SPLIT_TS
#define SPLIT_TS(n) \
    if (g == 0 && (n) < 16) tsv[(n)] = __builtin_amdgcn_s_memrealtime()
#else
#define SPLIT_TS(n)
#endif

template <int BG>
constexpr int split_rows() { return BGT<BG>::KC + kSmallPlanH<BG>.ncore; }   // scratch rows of Zc doubles

using g_f64 = __attribute__((address_space(1))) double;
using g_u32 = __attribute__((address_space(1))) uint32_t;

// hand-off loads / stores: global (not flat) sc1 accesses
__device__ __forceinline__ double ld_sc1(const double* base, uint32_t byte) {
    return __hip_atomic_load((g_f64*)((uintptr_t)base + byte), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* base, uint32_t byte, double v) {
    __hip_atomic_store((g_f64*)((uintptr_t)base + byte), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load((g_u32*)(uintptr_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Work split.  A wave owns one CHUNK: 64 consecutive slots z of one base row (phase A) and of one
// core column (phase B), so a row's / column's degree is wave-uniform and a wave issues exactly its
// edges' loads.  The chunks are dealt to the W workgroups in degree-descending order, snake-wise
// (wave v of workgroup w takes chunk v*W + w, or v*W + W-1-w for odd v), so every workgroup moves
// about the same number of bytes per phase: the barriers wait for the slowest workgroup, and a
// CU's remote-load bandwidth, not its ALUs, bounds a phase (measured r05: with rows / columns in
// natural order workgroup 0 alone held the degree-19 rows and the degree-30 column).
template <int BG>
struct SplitPlan {
    int8_t rord[BGT<BG>::MB] = {};   // base rows, degree descending (ties: ascending index)
    int8_t cord[BGT<BG>::KC] = {};   // core columns, degree descending
    constexpr SplitPlan() {
        using P = BGT<BG>;
        bool used[P::MB] = {};
        for (int n = 0; n < P::MB; ++n) {
            int b = -1;
            for (int i = 0; i < P::MB; ++i)
                if (!used[i] && (b < 0 || P::RS[i + 1] - P::RS[i] > P::RS[b + 1] - P::RS[b])) b = i;
            used[b] = true, rord[n] = (int8_t)b;
        }
        bool cu[P::KC] = {};
        constexpr SmallPlan<BG> sp{};
        for (int n = 0; n < P::KC; ++n) {
            int b = -1;
            for (int j = 0; j < P::KC; ++j)
                if (!cu[j] && (b < 0 || sp.cstart[j + 1] - sp.cstart[j] > sp.cstart[b + 1] - sp.cstart[b])) b = j;
            cu[b] = true, cord[n] = (int8_t)b;
        }
    }
};
template <int BG>
__device__ constexpr SplitPlan<BG> kSplitPlanD{};

// a codeblock's sync words back to zero (sc1 vector stores; the next split launch of the device
// starts after this kernel ends — the launcher's chain)
__device__ inline void sync_clear(uint32_t* sy) {
    for (int k = 0; k < 4; ++k)
        __hip_atomic_store((g_u32*)(uintptr_t)(sy + k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// R chunks per wave (R = 2 halves the workgroups per codeblock, so twice as many codeblocks fit
// one launch): wave v of workgroup w owns chunks of rounds v*R .. v*R + R-1, each round dealt
// snake-wise as above; the chunks of a wave are walked one after the other in each phase.
template <int BG, bool OFS, int R>
__global__ __launch_bounds__(kSplitThreads) void ldpc_split_kernel(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int Zc, int zi, int W, int64_t ldl, int64_t ldc, int L, double alpha,
    double beta, int pc, double* __restrict__ scratch, uint32_t* __restrict__ sync,
    uint32_t* __restrict__ ticket) {
    using P = BGT<BG>;
    using T = double;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, TS = 8;
    constexpr int DMAX = kSmallPlanH<BG>.dmax, CMAX = kSmallPlanH<BG>.cmax;
    // loads in flight per chunk (phase A, B); R = 2 keeps twice the chunk state, so fewer
    constexpr int CH = R == 1 ? LDPC5G_SPLIT_CH : 16, CCH = R == 1 ? LDPC5G_SPLIT_CCH : 16;
    __shared__ uint32_t rws[MB * DMAX], wws[MB * DMAX];   // edge words per (row, edge < DMAX)
    __shared__ uint32_t lfail, lflag, lticket, labort;

    const int t = threadIdx.x, lane = t & 63;
    const int v = __builtin_amdgcn_readfirstlane(t >> 6);
#ifdef LDPC5G_SPLIT_TS
    uint64_t tsv[16] = {};
#endif
    const int g = blockIdx.x * kSplitThreads + t;   // (instrumentation: workgroup 0, thread 0)
    SPLIT_TS(0);
    // (codeblock, part) by arrival ticket, not by blockIdx: the parts of a codeblock go to
    // workgroups that are resident, so at most one codeblock of the launch has some of its parts
    // waiting for CUs while the others run to completion and free theirs — two processes sharing
    // the GPU cannot each hold part of the chip waiting for the rest.  The ticket is taken here and
    // read after the edge-word fill (its round trip overlaps it).
    uint32_t tk = 0u;
    if (t == 0) tk = __hip_atomic_fetch_add((g_u32*)(uintptr_t)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ZT = (uint32_t)(Zc * TS);

    // ---- edge words: read word = column byte offset | (V mod Zc)*8 << 17; write word = CSC slot
    //      byte offset | (V mod Zc)*8 << 20
    for (int q = t; q < MB * DMAX; q += kSplitThreads) {
        const int i = q / DMAX, x = q - i * DMAX;
        const int e0 = row_start_d<BG>(i), dc = row_start_d<BG>(i + 1) - e0 - (i >= 4 ? 1 : 0);
        uint32_t rw = 0u, ww = 0u;
        if (x < dc) {
            const uint32_t w0 = kSmallPlanD<BG>.ew[e0 + x];
            const uint32_t sb = (uint32_t)shift_of<BG>(zi, e0 + x) * TS;
            rw = (w0 & 0xffu) * ZT | (sb << 17);
            ww = (w0 >> 8) * ZT | (sb << 20);
        }
        rws[q] = rw, wws[q] = ww;
    }
    if (t == 0) {
        // the last ticket of the launch: every workgroup holds its own, the counter goes back to 0
        if (tk == gridDim.x - 1u)
            __hip_atomic_store((g_u32*)(uintptr_t)ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lticket = tk, lfail = 0u, labort = 0u;
    }
    __syncthreads();
    const int tkt = __builtin_amdgcn_readfirstlane((int)lticket);
    const int cb = tkt / W, w = tkt - cb * W;
    const T* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    double* lq = scratch + (size_t)cb * split_rows<BG>() * Zc;   // [KC][Zc] LQ of the core columns
    double* msg = lq + (size_t)KC * Zc;                            // [NCE][Zc] messages, CSC slots
    uint32_t* sy = sync + cb * kSplitSync;   // [0] barrier counter, [1] fail tag, [2] final fail, [3] exits
    uint32_t* timeouts = ticket + 1;         // the device's count of timed-out codeblocks

    // barrier over the codeblock's W workgroups.  sig: this workgroup's fail tag (LDS lfail) is
    // raised into sy[fi] first; afterwards lflag = sy[fi] for every thread of the workgroup.
    // Returns false when the codeblock was aborted (kSplitTimeoutTicks): the caller returns.
    uint32_t nbar = 0;
    auto grid_sync = [&](int fi, uint32_t sig) -> bool {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's hand-off stores done
        __syncthreads();
        nbar += (uint32_t)W;
        if (t == 0) {
            if (sig != 0u && lfail == sig) {
                __hip_atomic_fetch_max((g_u32*)(uintptr_t)(sy + fi), sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_fetch_add((g_u32*)(uintptr_t)sy, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t c;
            while ((c = ld_sc1(sy)) < nbar) {   // an aborted counter (bit 31) ends the wait too
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > kSplitTimeoutTicks) {
                    __hip_atomic_fetch_or((g_u32*)(uintptr_t)sy, kSplitAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    c = kSplitAbort;
                    break;
                }
            }
            labort = c & kSplitAbort;
            lflag = ld_sc1(sy + fi);
        }
        __syncthreads();
        if (labort == 0u) return true;
        if (t == 0) {   // every part ends up here once: the last one out counts and cleans up
            status[cb] = 0, iters[cb] = -1;
            if (__hip_atomic_fetch_add((g_u32*)(uintptr_t)(sy + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (uint32_t)(W - 1)) {
                __hip_atomic_fetch_add((g_u32*)(uintptr_t)timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sync_clear(sy);
            }
        }
        return false;
    };

    const int nch = (Zc + 63) >> 6;   // chunks per row / column
    // per chunk slot k < R: own core column entry (cj, cz) and own check node (ri, rz)
    int cj[R], cn[R], ri[R], rd[R], dc[R], cz[R], rz[R];
    uint32_t cr0[R], cq[R], zb0[R], re0[R], wd[R];
    bool hasc[R], cpun[R], hasn[R], xe[R], hdx[R];
    T lf[R], lqv[R], xl[R], nA[R], nB[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int round = v * R + k;
        const int ch = round * W + ((round & 1) ? W - 1 - w : w);   // chunk (rank in degree order)
        const bool hasc_w = ch < KC * nch;
        cj[k] = hasc_w ? kSplitPlanD<BG>.cord[ch / nch] : 0;
        cz[k] = (ch % nch) * 64 + lane;
        hasc[k] = hasc_w && cz[k] < Zc;
        cn[k] = kSmallPlanD<BG>.cstart[cj[k] + 1] - kSmallPlanD<BG>.cstart[cj[k]];
        cr0[k] = (uint32_t)kSmallPlanD<BG>.cstart[cj[k]] * ZT + (uint32_t)cz[k] * TS;
        cq[k] = (uint32_t)cj[k] * ZT + (uint32_t)cz[k] * TS;   // LQ entry
        cpun[k] = cj[k] < pc;
        lf[k] = (hasc[k] && !cpun[k]) ? lrow[(cj[k] - pc) * Zc + cz[k]] : T(0);
        lqv[k] = lf[k];
        if (hasc[k]) st_sc1(lq, cq[k], lf[k]);
        const bool hasn_w = ch < MB * nch;
        ri[k] = hasn_w ? kSplitPlanD<BG>.rord[ch / nch] : 0;
        rz[k] = (ch % nch) * 64 + lane;
        hasn[k] = hasn_w && rz[k] < Zc;
        zb0[k] = (uint32_t)rz[k] * TS, re0[k] = (uint32_t)(ri[k] * DMAX);
        rd[k] = row_start_d<BG>(ri[k] + 1) - row_start_d<BG>(ri[k]);
        xe[k] = ri[k] >= 4;   // rows >= 4: the last edge is the extension column
        dc[k] = rd[k] - (xe[k] ? 1 : 0);
        xl[k] = (hasn[k] && xe[k]) ? lrow[(KB + ri[k] - pc) * Zc + rz[k]] : T(0);
        nA[k] = T(0), nB[k] = T(0), wd[k] = 0u, hdx[k] = false;
    }
    uint32_t mv = 0x80000000u;
    asm volatile("" : "+v"(mv));
    // iteration 0's phase A reads LQ_0 = the LLRs straight from the input (punctured columns 0), so
    // no barrier is needed before it; only L = 0 reads the scratch LQ (the final pass) right away
    if (L == 0 && !grid_sync(1, 0u)) return;
    SPLIT_TS(1);
    const uint32_t pcZT = (uint32_t)pc * ZT;
    const char* lrowb = (const char*)lrow - pcZT;   // byte offset col*ZT + z*8 of LQ_0 (col >= pc)

    int it = 0;
    for (; it < L; ++it) {
        // ---- phase A (rows from LQ_old, syndrome of LQ_old): each chunk's row, its dc core edges
        bool fail = false;
        auto phase_a = [&](auto firstc) {
        constexpr bool FIRST = decltype(firstc)::value;
        sfor<0, R>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            // per-iteration opaque copy: the addresses are loop-invariant, and hoisting them out of
            // the iteration loop (~40 extra live VGPRs) spills
            uint32_t zb = zb0[k];
            asm volatile("" : "+v"(zb));
            if (hasn[k]) {
                const int d = rd[k], dck = dc[k];
                const uint32_t rb = re0[k];
                uint32_t u = wd[k] << (32 - d);
                const uint32_t idxo = wd[k] >> 24;
                const T mA = nA[k], mB = nB[k];
                T min1 = FT<T>::inf(), min2 = FT<T>::inf();
                uint32_t idx = 0, negs = 0;
                bool par = false;
                auto edge = [&](uint32_t q0, T av, T rold) {
                    par ^= av < T(0);
                    const T q = av - rold;
                    const T aq = fabs(q);
                    idx = aq < min1 ? q0 : idx;
                    asm volatile("" : "+v"(idx));
                    negs = __builtin_amdgcn_alignbit(negs, FT<T>::sbits(q), 31);
                    two_min(min1, min2, aq);
                };
                // the row's LQ reads CH at a time, a chunk's all in flight before the first is used
                sfor<0, (DMAX + CH - 1) / CH>([&](auto cc) {
                    constexpr int c0 = decltype(cc)::value * CH, c1 = c0 + CH < DMAX ? c0 + CH : DMAX;
                    if (c0 < dck) {
                        T a[CH];
                        sfor<c0, c1>([&](auto xc) {
                            constexpr int x = decltype(xc)::value;
                            if (x < dck) {
                                const uint32_t Wx = rws[rb + x];
                                const uint32_t zz = zb + (Wx >> 17);
                                const uint32_t off = (Wx & 0x1ffffu) + min(zz, zz - ZT);
                                if constexpr (FIRST)
                                    a[x - c0] = off >= pcZT ? *(const g_f64*)(uintptr_t)(lrowb + off) : T(0);
                                else
                                    a[x - c0] = ld_sc1(lq, off);
                            }
                        });
                        sfor<c0, c1>([&](auto xc) {
                            constexpr int x = decltype(xc)::value;
                            if (x < dck) {
                                const T rold = xsign_v(idxo == (uint32_t)x ? mB : mA, u, mv);
                                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1
                                edge((uint32_t)x, a[x - c0], rold);
                            }
                        });
                    }
                });
                if (xe[k]) {   // the extension edge (the row's last): LQ of the degree-1 column = LLR + its r
                    const T rold = xsign_v(idxo == (uint32_t)dck ? mB : mA, wd[k] << 31, mv);
                    const T av = xl[k] + rold;
                    hdx[k] = av < T(0);
                    edge((uint32_t)dck, av, rold);
                }
                fail |= par;
                T x1 = min1, x2 = min2;
                if constexpr (OFS) {
                    x1 = min1 - beta, x2 = min2 - beta;   // max(minv - beta, 0) (:201)
                    x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
                }
                const uint32_t sgn = 0u - (__builtin_popcount(negs) & 1u);   // row sign product
                const uint32_t flip = sgn & ((1u << d) - 1u);
                const T nAk = alpha * x1, nBk = alpha * x2;
                nA[k] = nAk, nB[k] = nBk;
                wd[k] = (negs ^ flip) | (idx << 24);
                uint32_t un = wd[k] << (32 - d);
                sfor<0, DMAX>([&](auto xc) {
                    constexpr int x = decltype(xc)::value;
                    if (x < dck) {
                        const uint32_t V = wws[rb + x];
                        const T r = xsign_v(idx == (uint32_t)x ? nBk : nAk, un, mv);
                        asm("v_add_u32 %0, %1, %1" : "=v"(un) : "v"(un));
                        const uint32_t zz = zb + (V >> 20);
                        st_sc1(msg, (V & 0xfffffu) + min(zz, zz - ZT), r);
                    }
                });
            }
        });
        };
        if (it == 0)
            phase_a(std::true_type{});
        else
            phase_a(std::false_type{});
        if (fail) lfail = (uint32_t)(it + 1);
        if (it < 2) SPLIT_TS(2 + 4 * it);
        if (!grid_sync(1, (uint32_t)(it + 1))) return;
        if (it < 2) SPLIT_TS(3 + 4 * it);
        if (lflag != (uint32_t)(it + 1)) {
            // ---- the syndrome of LQ_old holds (:112-114): its hard decisions are the output
#pragma unroll
            for (int k = 0; k < R; ++k) {
                if (hasc[k]) crow[cj[k] * Zc + cz[k]] = (int8_t)(lqv[k] < T(0));
                if (hasn[k] && xe[k]) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)hdx[k];
            }
            if (w == 0 && t == 0) status[cb] = 1, iters[cb] = it;
            // the sync words go back to zero for the next launch: the last workgroup to leave (every
            // one has read sy[1] by now) clears them
            if (t == 0 && __hip_atomic_fetch_add((g_u32*)(uintptr_t)(sy + 3), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(W - 1))
                sync_clear(sy);
            return;
        }
        // ---- phase B: LQ = LLRin + Lr.sum(axis=0) (:126), rows ascending: each chunk's column
        sfor<0, R>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            uint32_t cr = cr0[k];
            asm volatile("" : "+v"(cr));
            if (hasc[k]) {
                const int n = cn[k];
                T acc = T(0);
                sfor<0, (CMAX + CCH - 1) / CCH>([&](auto cc) {
                    constexpr int p0 = decltype(cc)::value * CCH, p1 = p0 + CCH < CMAX ? p0 + CCH : CMAX;
                    if (p0 < n) {
                        T m[CCH];
                        sfor<p0, p1>([&](auto pc_) {
                            constexpr int p = decltype(pc_)::value;
                            if (p < n) m[p - p0] = ld_sc1(msg, cr + (uint32_t)p * ZT);
                        });
                        sfor<p0, p1>([&](auto pc_) {
                            constexpr int p = decltype(pc_)::value;
                            if (p < n) acc = acc + m[p - p0];
                        });
                    }
                });
                lqv[k] = (cpun[k] ? T(0) : lf[k]) + acc;   // punctured columns: LLR 0 (:43)
                st_sc1(lq, cq[k], lqv[k]);
            }
        });
        if (it < 2) SPLIT_TS(4 + 4 * it);
        if (!grid_sync(1, 0u)) return;
        if (it < 2) SPLIT_TS(5 + 4 * it);
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    SPLIT_TS(10);
    bool ox[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        ox[k] = false;
        if (hasn[k]) {
            bool par = false;
            const int dck = dc[k];
            if (xe[k]) {
                const T rx = xsign_v((wd[k] >> 24) == (uint32_t)dck ? nB[k] : nA[k], wd[k] << 31, mv);
                ox[k] = xl[k] + rx <= T(0);
                par = ox[k];
            }
            sfor<0, DMAX>([&](auto xc) {
                constexpr int x = decltype(xc)::value;
                if (x < dck) {
                    const uint32_t Wx = rws[re0[k] + x];
                    const uint32_t zz = zb0[k] + (Wx >> 17);
                    par ^= ld_sc1(lq, (Wx & 0x1ffffu) + min(zz, zz - ZT)) <= T(0);
                }
            });
            if (par) lfail = (uint32_t)(L + 1);
        }
    }
    SPLIT_TS(11);
    // ---- the decisions need no barrier; the status does: every workgroup raises its fail flag and
    //      then adds to the counter, and the workgroup whose add comes last (told by the value the
    //      add returns) reads the flag and writes the status — nobody waits
#pragma unroll
    for (int k = 0; k < R; ++k) {
        if (hasc[k]) crow[cj[k] * Zc + cz[k]] = (int8_t)(lqv[k] <= T(0));
        if (hasn[k] && xe[k]) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)ox[k];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        if (lfail == (uint32_t)(L + 1)) {
            __hip_atomic_fetch_max((g_u32*)(uintptr_t)(sy + 2), (uint32_t)(L + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t old = __hip_atomic_fetch_add((g_u32*)(uintptr_t)sy, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == nbar + (uint32_t)W) status[cb] = ld_sc1(sy + 2) == 0u, iters[cb] = L, sync_clear(sy);
    }
    SPLIT_TS(12);
#ifdef LDPC5G_SPLIT_TS
    SPLIT_TS(13);
    __syncthreads();
    if (g == 0) for (int q_ = 0; q_ < 16; ++q_) ((uint64_t*)crow)[q_] = tsv[q_];
#endif
}

// per-device state of the split launches (both base graphs): the chain event, the sync area
// (kSplitMaxWG codeblock lines + the ticket line: [0] ticket, [1] timed-out codeblocks), the scratch
struct SplitState {
    std::mutex mu;
    hipEvent_t last[64] = {};
    uint32_t* sync[64] = {};
    void* scratch[64] = {};
    size_t cap[64] = {};
};
SplitState& split_state() {
    static SplitState s;
    return s;
}

template <int BG>
int launch_split_t(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                   int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                   hipStream_t st) {
    const int R = split_wanted(BG, B, Zc);
    if (R == 0) return fail(LDPC5G_ESIZE, "split decoder: %d codeblocks of Zc=%d do not fit", B, Zc);
    const int W = split_parts(BG, Zc, R);
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (dev < 0 || dev >= 64) return fail(LDPC5G_ESIZE, "device ordinal %d >= 64", dev);
    const size_t bytes = (size_t)B * split_rows<BG>() * Zc * sizeof(double);
    int rc = 0;
    {
        // split launches of one device run one after another, whatever their streams and base
        // graphs (a per-device event chain; on one stream it costs nothing), so they share one
        // scratch and one sync area per device, plain hipMalloc memory (the hand-off table's row):
        // the scratch grows on demand (after the previous launch has ended), the sync area is
        // zeroed once and every launch leaves its words zero again (sync_clear), so no allocation
        // or memset runs per call
        SplitState& S = split_state();
        std::lock_guard<std::mutex> lk(S.mu);
        hipEvent_t& ev = S.last[dev];
        uint32_t*& sync = S.sync[dev];
        void*& p = S.scratch[dev];
        if (!sync) {
            const size_t sb = ((size_t)kSplitMaxWG + 1) * kSplitSync * 4;   // + the ticket line
            void* q = nullptr;
            rc = check_hip(hipMalloc(&q, sb), "hipMalloc (split sync area)");
            if (!rc) rc = check_hip(hipMemset(q, 0, sb), "hipMemset (split sync area)");
            if (!rc) rc = check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize (split sync area)");
            if (!rc) sync = (uint32_t*)q;
        }
        if (!rc && S.cap[dev] < bytes) {
            if (p) {
                if (ev) rc = check_hip(hipEventSynchronize(ev), "hipEventSynchronize (split scratch)");
                if (!rc) rc = check_hip(hipFree(p), "hipFree (split scratch)");
                p = nullptr, S.cap[dev] = 0;
            }
            // at least 24 BG1 Zc = 384 codeblocks' worth (20 MB), so most devices allocate once
            const size_t want = std::max(bytes, (size_t)24 * split_rows<1>() * 384 * sizeof(double));
            if (!rc) rc = check_hip(hipMalloc(&p, want), "hipMalloc (split scratch)");
            if (!rc) S.cap[dev] = want;
        }
        if (rc) {
        } else if (!ev) {
            rc = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate (split chain)");
        } else {
            rc = check_hip(hipStreamWaitEvent(st, ev, 0), "hipStreamWaitEvent (split chain)");
        }
        if (!rc) {
            auto kern = R == 1 ? (beta != 0.0 ? ldpc_split_kernel<BG, true, 1> : ldpc_split_kernel<BG, false, 1>)
                               : (beta != 0.0 ? ldpc_split_kernel<BG, true, 2> : ldpc_split_kernel<BG, false, 2>);
            hipLaunchKernelGGL(kern, dim3(B * W), dim3(kSplitThreads), 0, st, llr, ck, status, iters, Zc, zi, W,
                               ldl, ldc, L, alpha, beta, pc, (double*)p, sync, sync + kSplitMaxWG * kSplitSync);
            rc = check_hip(hipGetLastError(), "ldpc_split_kernel launch");
            if (!rc) rc = check_hip(hipEventRecord(ev, st), "hipEventRecord (split chain)");
        }
    }
    return rc;
}

}  // namespace

int split_parts(int bgn, int Zc, int R) {   // 64-slot row chunks, R per wave, 16-wave workgroups
    const int mb = bgn == 1 ? BGT<1>::MB : BGT<2>::MB;
    const int per = R * (kSplitThreads / 64);
    return (mb * ((Zc + 63) / 64) + per - 1) / per;
}

int split_wanted(int bgn, int B, int Zc) {
    // LDPC5G_NO_SPLIT=1: the one-workgroup-per-codeblock kernels instead (A/B measurements)
    static const bool off = [] { const char* e = getenv("LDPC5G_NO_SPLIT"); return e && *e && *e != '0'; }();
    // BG2 Zc <= 64 keeps the small-codeblock kernel (its LDS image fits one CU)
    if (off || B < 1 || Zc < 64 || (bgn == 2 && Zc <= 64)) return 0;
    // the launch fills at most 7/8 of the device's CUs (224 of 256; a partitioned device has fewer),
    // and a codeblock's W workgroups must fit the device at once
    static std::atomic<int> cus_of[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev < 0 || dev >= 64) return 0;   // (the split launcher refuses such devices)
    int cus = cus_of[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 0;
        cus_of[dev].store(cus, std::memory_order_relaxed);
    }
    const int maxwg = std::min(kSplitMaxWG, cus * 7 / 8);
    const int w1 = split_parts(bgn, Zc, 1), w2 = split_parts(bgn, Zc, 2);
    if (w1 <= cus && B * w1 <= maxwg) return 1;
    if (w2 <= cus && B * w2 <= maxwg) return 2;
    return 0;
}

int split_timeouts(uint32_t* count) {
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (dev < 0 || dev >= 64) return fail(LDPC5G_ESIZE, "device ordinal %d >= 64", dev);
    SplitState& S = split_state();
    std::lock_guard<std::mutex> lk(S.mu);
    *count = 0;
    if (!S.sync[dev]) return LDPC5G_OK;   // no split launch on this device yet
    if (S.last[dev])
        if (int rc = check_hip(hipEventSynchronize(S.last[dev]), "hipEventSynchronize (split chain)")) return rc;
    return check_hip(hipMemcpy(count, S.sync[dev] + kSplitMaxWG * kSplitSync + 1, sizeof(uint32_t),
                               hipMemcpyDeviceToHost), "hipMemcpy (split timeouts)");
}

int launch_flood_split(int bgn, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                       int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta,
                       int pc, hipStream_t st) {
    return bgn == 1 ? launch_split_t<1>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_split_t<2>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
