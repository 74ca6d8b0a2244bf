// ldpc5g_capi.hip — the extern "C" boundary of libldpc5g.so (include/ldpc5g.h): argument
// validation, error codes, mixed-batch work lists; kernels live in ldpc5g_{enc,dec,bfbp}.hip.
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

void clear_error() { g_err.clear(); }

const char* err_text() { return g_err.c_str(); }

int zc_index(int Zc) {
    for (int i = 0; i < LDPC5G_NUM_ZC; ++i)
        if (kLdpcZcList[i] == Zc) return i;
    return -1;
}

int check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(LDPC5G_EHIP, "%s: %s", what, hipGetErrorString(e));
    return LDPC5G_OK;
}

namespace {
// Pinned staging pool for small host-built plans (stage_h2d).  A hipMemcpyAsync from pageable
// memory may return before the runtime has read the source, so plans are first copied into a
// pinned slot; a slot is reused only after the event recorded behind its copy has completed.
// The pool grows (up to kMaxSlots per thread) instead of waiting: a caller that queues many
// decodes ahead of the GPU is throttled only past kMaxSlots plans in flight.  The slots are held
// per thread for the life of the process, never freed (a thread-exit destructor could run after
// the HIP runtime is gone); include/ldpc5g.h states it.
struct PinnedSlot {
    void* buf = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    int dev = -1;
    bool pending = false;
};
constexpr size_t kMaxSlots = 64;
thread_local std::vector<PinnedSlot>* t_pool = nullptr;   // leaked on purpose (see above)
thread_local size_t t_next = 0;

// a free slot: one whose copy has completed (non-blocking query), else a new one, else wait for
// the oldest-issued (round-robin) slot
int take_slot(PinnedSlot** out) {
    if (!t_pool) t_pool = new std::vector<PinnedSlot>();
    std::vector<PinnedSlot>& pool = *t_pool;
    for (size_t k = 0; k < pool.size(); ++k) {
        PinnedSlot& s = pool[(t_next + k) % pool.size()];
        if (s.pending && hipEventQuery(s.ev) == hipSuccess) s.pending = false;
        if (!s.pending) {
            t_next = (t_next + k + 1) % pool.size();
            *out = &s;
            return LDPC5G_OK;
        }
    }
    if (pool.size() < kMaxSlots) {
        pool.emplace_back();
        *out = &pool.back();
        return LDPC5G_OK;
    }
    PinnedSlot& s = pool[t_next];
    t_next = (t_next + 1) % pool.size();
    if (int rc = check_hip(hipEventSynchronize(s.ev), "hipEventSynchronize(staging)")) return rc;
    s.pending = false;
    *out = &s;
    return LDPC5G_OK;
}
}  // namespace

int stage_h2d(void* dst, const void* src, size_t n, hipStream_t st) {
    if (n == 0) return LDPC5G_OK;
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    PinnedSlot* sp = nullptr;
    if (int rc = take_slot(&sp)) return rc;
    PinnedSlot& s = *sp;
    if (s.dev != dev && s.ev) {
        (void)hipEventDestroy(s.ev);
        s.ev = nullptr;
    }
    if (!s.ev) {
        if (int rc = check_hip(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate(staging)")) return rc;
        s.dev = dev;
    }
    if (s.cap < n) {
        if (s.buf) (void)hipHostFree(s.buf);
        s.buf = nullptr, s.cap = 0;
        const size_t cap = std::max<size_t>(n, 4096);
        if (int rc = check_hip(hipHostMalloc(&s.buf, cap, hipHostMallocDefault), "hipHostMalloc(staging)")) return rc;
        s.cap = cap;
    }
    memcpy(s.buf, src, n);
    if (int rc = check_hip(hipMemcpyAsync(dst, s.buf, n, hipMemcpyHostToDevice, st), "hipMemcpyAsync(plan)")) return rc;
    if (int rc = check_hip(hipEventRecord(s.ev, st), "hipEventRecord(staging)")) return rc;
    s.pending = true;
    return LDPC5G_OK;
}

namespace {
// Mixed-batch plan layout (host bytes, copied verbatim to the device):
//   MixedPlanHdr | DecWork[nw1] (BG1) | DecWork[nw2] (BG2) | CbRef[nref]
struct MixedPlanHdr {
    int32_t magic, schedule, nw1, nw2, nref;
    int32_t nz1;   // the last nz1 BG1 work items: Zc = 384 with a full G (the Zc = 384 kernels)
    int32_t nz2;   // the same for BG2 (float64 flooding: the frame kernel)
    int32_t pad;   // 32 bytes: the CbRef array after the work items stays 8-byte aligned
};
static_assert(sizeof(MixedPlanHdr) == 32 && sizeof(DecWork) % 8 == 0, "plan layout");
constexpr int32_t kPlanMagic = 0x4c504d58;   // "XMPL"

int64_t build_plan(const ldpc5g_cb_desc_t* desc, int B, int schedule, void* out, int64_t cap) {
    // group codeblocks by (bgn, Zc), pack G = floor(threads/Zc) per workgroup
    std::vector<std::vector<int>> bucket[2];
    bucket[0].resize(LDPC5G_NUM_ZC);
    bucket[1].resize(LDPC5G_NUM_ZC);
    for (int b = 0; b < B; ++b) {
        const ldpc5g_cb_desc_t& d = desc[b];
        if (d.bgn != 1 && d.bgn != 2) return fail(LDPC5G_EBGN, "desc[%d]: bgn must be 1 or 2 (got %d)", b, d.bgn);
        const int zi = zc_index(d.Zc);
        if (zi < 0) return fail(LDPC5G_EZC, "desc[%d]: Zc=%d is not a lifting size", b, d.Zc);
        if (d.llr_off < 0 || d.ck_off < 0) return fail(LDPC5G_ESIZE, "desc[%d]: negative offset", b);
        bucket[d.bgn - 1][zi].push_back(b);
    }
    std::vector<DecWork> work[2];
    std::vector<CbRef> refs;
    int nz1 = 0, nz2 = 0;
    bool span_err = false;
    constexpr int kMaxN = 68 * 384;   // the longest codeblock row
    // lifting sizes ascending: the dispatcher hands workgroups to CUs in list order, and the
    // longest-running ones come first — a small-Zc workgroup holds G = 768 / Zc codeblocks (64 at
    // Zc = 12) and runs until its slowest one stops, nearly always all L iterations, while a
    // Zc = 384 workgroup (2 codeblocks) often exits early (r05 config 4: 0.951 ms per decode vs
    // 0.965 with lifting sizes descending).  Per bucket a partial workgroup first, then the full
    // ones: BG1's full Zc = 384 workgroups are the tail of its list (their own kernel, see below).
    for (int g = 0; g < 2; ++g)
        for (int zi = 0; zi < LDPC5G_NUM_ZC; ++zi) {
            const std::vector<int>& v = bucket[g][zi];
            const int Zc = kLdpcZcList[zi], G = dec_G(Zc, schedule == LDPC5G_LAYERED);
            const size_t part = v.size() % G;
            auto emit = [&](size_t s, int n) {
                DecWork w;
                w.zi = zi, w.Zc = Zc, w.G = n, w.first = (int)refs.size();
                for (int c = 0; c < n; ++c) {
                    CbRef r;
                    r.llr_off = desc[v[s + c]].llr_off, r.ck_off = desc[v[s + c]].ck_off, r.out = v[s + c], r.pad = 0;
                    refs.push_back(r);
                }
                // a work item's codeblocks by LLR offset: the first is the lowest, the base of the
                // layered kernel's 32-bit lane offsets (ldpc5g_dec_body.h), whose span is checked
                std::sort(refs.begin() + w.first, refs.end(),
                          [](const CbRef& a, const CbRef& b) { return a.llr_off < b.llr_off; });
                if ((refs.back().llr_off - refs[w.first].llr_off + (int64_t)kMaxN) * 8 >= ((int64_t)1 << 32))
                    span_err = true;
                work[g].push_back(w);
            };
            if (part) emit(0, (int)part);
            for (size_t s = part; s < v.size(); s += G) emit(s, G);
            if (Zc == 384) (g == 0 ? nz1 : nz2) = (int)((v.size() - part) / G);
        }
    if (span_err) return fail(LDPC5G_ESIZE, "a work item's codeblock LLR rows span >= 4 GiB (rows of one (bgn, Zc) too far apart)");
    const int64_t need = (int64_t)sizeof(MixedPlanHdr) + (int64_t)(work[0].size() + work[1].size()) * (int64_t)sizeof(DecWork) +
                         (int64_t)refs.size() * (int64_t)sizeof(CbRef);
    if (!out || cap < need) return need;
    unsigned char* p = (unsigned char*)out;
    MixedPlanHdr h{kPlanMagic, schedule, (int32_t)work[0].size(), (int32_t)work[1].size(), (int32_t)refs.size(), nz1,
                   nz2, 0};
    memcpy(p, &h, sizeof h);
    p += sizeof h;
    for (int g = 0; g < 2; ++g) {   // (an empty vector's data() may be null: no memcpy from it)
        if (!work[g].empty()) memcpy(p, work[g].data(), work[g].size() * sizeof(DecWork));
        p += work[g].size() * sizeof(DecWork);
    }
    if (!refs.empty()) memcpy(p, refs.data(), refs.size() * sizeof(CbRef));
    return need;
}

// A second stream per (thread, device) for the BG2 half of a mixed plan: the BG1 and BG2 launches
// then share the GPU instead of running one after the other (each alone leaves a partly idle last
// round of workgroups).  Ordered against the caller's stream by two events; created once, never
// destroyed (like the staging buffers).
struct SideStream {
    hipStream_t s = nullptr, s2 = nullptr;   // s2: the Zc = 384 share of a mixed plan (LDPC5G_MIX_Z3)
    hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr;
};
thread_local SideStream t_side[64];

int side_stream(SideStream** out) {
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (dev < 0 || dev >= 64) return fail(LDPC5G_ESIZE, "device ordinal %d >= 64", dev);
    SideStream& x = t_side[dev];
    if (!x.s) {
        if (int rc = check_hip(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking), "hipStreamCreate(side)")) return rc;
        if (int rc = check_hip(hipEventCreateWithFlags(&x.fork, hipEventDisableTiming), "hipEventCreate(fork)")) return rc;
        if (int rc = check_hip(hipEventCreateWithFlags(&x.join, hipEventDisableTiming), "hipEventCreate(join)")) return rc;
        if (int rc = check_hip(hipStreamCreateWithFlags(&x.s2, hipStreamNonBlocking), "hipStreamCreate(side 2)")) return rc;
        if (int rc = check_hip(hipEventCreateWithFlags(&x.join2, hipEventDisableTiming), "hipEventCreate(join2)")) return rc;
    }
    *out = &x;
    return LDPC5G_OK;
}

// launches of a plan (host copy `h` for the counts, device copy `dev` for the kernels)
// BG1's full Zc = 384 work items on a third stream with the Zc = 384 kernel, however few (r05
// config 4: 171 of them, step 1.017 -> 1.004 ms, decode 0.938 -> 0.930); 0: only when >= 512 of
// them, in line on the caller's stream
#ifndef LDPC5G_MIX_Z3
#define LDPC5G_MIX_Z3 1
#endif
int launch_plan(const MixedPlanHdr& h, const unsigned char* dev, const void* llr_base, int llr_dtype,
                int8_t* ck_base, uint8_t* status, int32_t* iters, int L, double alpha, double beta,
                int pc, bool dead, hipStream_t st) {
    const DecWork* w1 = (const DecWork*)(dev + sizeof(MixedPlanHdr));
    const DecWork* w2 = w1 + h.nw1;
    const CbRef* r = (const CbRef*)(w2 + h.nw2);
    const bool lay = h.schedule == LDPC5G_LAYERED;
    // BG1's full Zc = 384 work items (the tail of its list) run the Zc = 384 kernels of mixed plans
    // (layered float32, flooding float64; a mixed plan's float32 flooding items keep the generic
    // kernel, BG2's float64 ones go to the frame kernel below) as their own
    // launch on a third stream beside the rest (LDPC5G_MIX_Z3; in line on the caller's stream they
    // paid only when they fill the GPU on their own: config 4's 171 workgroups measured 1.04 ->
    // 1.17 ms split off in line)
    constexpr int kZcSplitMin = LDPC5G_MIX_Z3 ? 1 : 512;
    const int nz = (lay || llr_dtype == LDPC5G_F64) && h.nz1 >= kZcSplitMin ? std::min(h.nz1, h.nw1) : 0;
    // BG2 on the side stream when both base graphs are present (forked from / joined into st)
    SideStream* side = nullptr;
    const bool z3 = LDPC5G_MIX_Z3 && nz > 0 && h.nw1 - nz > 0;   // the Zc = 384 share on a third stream
    if ((h.nw2 > 0 && h.nw1 > 0) || z3) {
        if (int rc = side_stream(&side)) return rc;
        if (int rc = check_hip(hipEventRecord(side->fork, st), "hipEventRecord(fork)")) return rc;
        if (int rc = check_hip(hipStreamWaitEvent(side->s, side->fork, 0), "hipStreamWaitEvent(fork)")) return rc;
    }
    // BG2's full Zc = 384 work items: the float64 frame kernel (ldpc5g_dec_frame.h), launched
    // before BG2's other work items on the same stream
    const int nzb = !lay && llr_dtype == LDPC5G_F64 ? std::min(h.nz2, h.nw2) : 0;
    for (int g = 0; g < 2; ++g) {
        const int nwg = g == 0 ? h.nw1 - nz : h.nw2 - nzb;
        hipStream_t sg = g == 1 && side ? side->s : st;
        if (g == 1 && nzb > 0)
            if (int rc = launch_dec_mixed(2, llr_dtype, lay, llr_base, ck_base, status, iters, nzb,
                                          w2 + (h.nw2 - nzb), r, L, alpha, beta, pc, dead, sg, true))
                return rc;
        if (nwg > 0)
            if (int rc = launch_dec_mixed(g + 1, llr_dtype, lay, llr_base, ck_base, status, iters, nwg,
                                          g == 0 ? w1 : w2, r, L, alpha, beta, pc, dead, sg))
                return rc;
        if (g == 0 && nz > 0) {
            hipStream_t sz = z3 ? side->s2 : st;
            if (z3)
                if (int rc = check_hip(hipStreamWaitEvent(sz, side->fork, 0), "hipStreamWaitEvent(fork 2)")) return rc;
            if (int rc = launch_dec_mixed(1, llr_dtype, lay, llr_base, ck_base, status, iters, nz,
                                          w1 + (h.nw1 - nz), r, L, alpha, beta, pc, dead, sz, true))
                return rc;
            if (z3) {
                if (int rc = check_hip(hipEventRecord(side->join2, sz), "hipEventRecord(join2)")) return rc;
                if (int rc = check_hip(hipStreamWaitEvent(st, side->join2, 0), "hipStreamWaitEvent(join2)")) return rc;
            }
        }
    }
    if (side && h.nw2 > 0) {
        if (int rc = check_hip(hipEventRecord(side->join, side->s), "hipEventRecord(join)")) return rc;
        if (int rc = check_hip(hipStreamWaitEvent(st, side->join, 0), "hipStreamWaitEvent(join)")) return rc;
    }
    return LDPC5G_OK;
}

int check_mixed_args(int32_t B, int32_t L, int32_t llr_dtype, int32_t schedule, double beta) {
    if (B < 0 || L < 0) return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d", B, L);
    if (llr_dtype != LDPC5G_F64 && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "bad llr dtype %d", llr_dtype);
    if (schedule != LDPC5G_FLOODING && schedule != LDPC5G_LAYERED) return fail(LDPC5G_ESIZE, "bad schedule %d", schedule);
    if (schedule == LDPC5G_LAYERED && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "layered schedule requires float32 LLRs");
    if (!(beta >= 0.0)) return fail(LDPC5G_ESIZE, "beta=%g: the offset must be >= 0 (nr_ldpc_decode.py:60)", beta);
    return LDPC5G_OK;
}
}  // namespace

}  // namespace ldpc5g_impl

using namespace ldpc5g_impl;

// ================================================================================== C ABI
extern "C" {

const char* ldpc5g_version(void) { return LDPC5G_VERSION; }

// Diagnostics (not part of the drop-in surface): decoder workgroups resident per CU.
int ldpc5g_dec_blocks_per_cu(int32_t bgn, int32_t llr_dtype, int32_t schedule) {
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn=%d", bgn);
    return dec_blocks_per_cu(bgn, llr_dtype, schedule == LDPC5G_LAYERED);
}

const char* ldpc5g_last_error(void) { return g_err.c_str(); }

int ldpc5g_split_timeouts(uint32_t* count) {
    clear_error();
    if (!count) return fail(LDPC5G_ESIZE, "null count");
    return split_timeouts(count);
}

int ldpc5g_find_ils(int32_t Zc) {
    int i = zc_index(Zc);
    return i < 0 ? 255 : kLdpcZcSet[i];
}

int ldpc5g_encode(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc, int64_t ldk,
                  int64_t ldn, void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int K = (bgn == 1 ? 22 : 10) * Zc, N = (bgn == 1 ? 66 : 50) * Zc;
    if (B < 0 || (B > 1 && (ldk < K || ldn < N))) return fail(LDPC5G_ESIZE, "bad sizes B=%d ldk=%lld ldn=%lld (K=%d N=%d)", B, (long long)ldk, (long long)ldn, K, N);
    if (B == 0) return LDPC5G_OK;
    if (!ck || !dn) return fail(LDPC5G_ESIZE, "null buffer");
    return launch_encode(ck, dn, B, bgn, Zc, zi, ldk, ldn, (hipStream_t)stream);
}

int ldpc5g_decode_ms(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L, double alpha,
                     double beta, int32_t schedule, int32_t flags, int64_t ldl, int64_t ldc,
                     void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    const int N = (bgn == 1 ? 66 : 50) * Zc + (2 - pc) * Zc, Nf = (bgn == 1 ? 68 : 52) * Zc;
    if (B < 0 || L < 0 || (B > 1 && (ldl < N || ldc < Nf)))
        return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d ldl=%lld ldc=%lld (N=%d Nf=%d)", B, L, (long long)ldl, (long long)ldc, N, Nf);
    if (llr_dtype != LDPC5G_F64 && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "bad llr dtype %d", llr_dtype);
    if (schedule != LDPC5G_FLOODING && schedule != LDPC5G_LAYERED) return fail(LDPC5G_ESIZE, "bad schedule %d", schedule);
    if (schedule == LDPC5G_LAYERED && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "layered schedule requires float32 LLRs");
    if (!(beta >= 0.0)) return fail(LDPC5G_ESIZE, "beta=%g: the offset must be >= 0 (nr_ldpc_decode.py:60)", beta);
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    return launch_dec(bgn, llr_dtype, schedule == LDPC5G_LAYERED, llr, ck, status, iters, B, Zc, zi,
                      ldl, ldc, L, alpha, beta, pc, (flags & LDPC5G_RATE_MATCHED) != 0, (hipStream_t)stream);
}

namespace ldpc5g_impl {
namespace {
// Per-thread device + pinned buffers of the host-buffer entry points, one set per device ordinal
// (a thread that alternates devices keeps and reuses each device's set; grown on demand, never
// freed: a thread-exit destructor could run after the HIP runtime is gone; include/ldpc5g.h states it).
struct HostStage {
    void* dev = nullptr;
    size_t dcap = 0;
    void* pin = nullptr;
    size_t pcap = 0;
};
constexpr int kMaxStageDevices = 64;
thread_local HostStage t_hs[kMaxStageDevices];

int host_stage(size_t bytes, unsigned char** d, unsigned char** p) {
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (dev < 0 || dev >= kMaxStageDevices) return fail(LDPC5G_ESIZE, "device ordinal %d >= %d", dev, kMaxStageDevices);
    HostStage& h = t_hs[dev];
    if (h.dcap < bytes) {
        if (h.dev) (void)hipFree(h.dev);
        h.dev = nullptr, h.dcap = 0;
        if (int rc = check_hip(hipMalloc(&h.dev, bytes), "hipMalloc(host stage)")) return rc;
        h.dcap = bytes;
    }
    if (h.pcap < bytes) {
        if (h.pin) (void)hipHostFree(h.pin);
        h.pin = nullptr, h.pcap = 0;
        if (int rc = check_hip(hipHostMalloc(&h.pin, bytes, hipHostMallocDefault), "hipHostMalloc(host stage)")) return rc;
        h.pcap = bytes;
    }
    *d = (unsigned char*)h.dev, *p = (unsigned char*)h.pin;
    return LDPC5G_OK;
}
// an error after the first copy was queued: drain the stream before returning, so the next call
// on this thread never rewrites (or frees) a pinned buffer a queued copy may still be reading
int drained(int rc, hipStream_t st) {
    if (rc) (void)hipStreamSynchronize(st);
    return rc;
}
size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
}  // namespace
}  // namespace ldpc5g_impl

int ldpc5g_decode_ms_host(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int32_t B,
                          int32_t bgn, int32_t Zc, int32_t L, double alpha, double beta, int32_t flags,
                          void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    const int N = (bgn == 1 ? 66 : 50) * Zc + (2 - pc) * Zc, Nf = (bgn == 1 ? 68 : 52) * Zc;
    if (B < 0 || L < 0) return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d", B, L);
    if (!(beta >= 0.0)) return fail(LDPC5G_ESIZE, "beta=%g: the offset must be >= 0 (nr_ldpc_decode.py:60)", beta);
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    const size_t nin = (size_t)B * N * sizeof(double), nck = (size_t)B * Nf;
    const size_t o_ck = align16(nin), o_st = align16(o_ck + nck), o_it = align16(o_st + B);
    const size_t total = o_it + (size_t)B * 4;
    unsigned char *d = nullptr, *p = nullptr;
    if (int rc = host_stage(total, &d, &p)) return rc;
    hipStream_t st = (hipStream_t)stream;
    memcpy(p, llr, nin);
    if (int rc = check_hip(hipMemcpyAsync(d, p, nin, hipMemcpyHostToDevice, st), "hipMemcpyAsync(llr)")) return drained(rc, st);
    if (int rc = launch_dec(bgn, LDPC5G_F64, false, d, (int8_t*)(d + o_ck), d + o_st, (int32_t*)(d + o_it), B, Zc, zi,
                            N, Nf, L, alpha, beta, pc, (flags & LDPC5G_RATE_MATCHED) != 0, st))
        return drained(rc, st);
    if (int rc = check_hip(hipMemcpyAsync(p + o_ck, d + o_ck, total - o_ck, hipMemcpyDeviceToHost, st), "hipMemcpyAsync(out)"))
        return drained(rc, st);
    if (int rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize")) return rc;
    memcpy(ck, p + o_ck, nck);
    memcpy(status, p + o_st, (size_t)B);
    memcpy(iters, p + o_it, (size_t)B * 4);
    return LDPC5G_OK;
}

int ldpc5g_encode_host(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc, void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int K = (bgn == 1 ? 22 : 10) * Zc, N = (bgn == 1 ? 66 : 50) * Zc;
    if (B < 0) return fail(LDPC5G_ESIZE, "bad size B=%d", B);
    if (B == 0) return LDPC5G_OK;
    if (!ck || !dn) return fail(LDPC5G_ESIZE, "null buffer");
    const size_t nk = (size_t)B * K, o_dn = align16(nk), total = o_dn + (size_t)B * N;
    unsigned char *d = nullptr, *p = nullptr;
    if (int rc = host_stage(total, &d, &p)) return rc;
    hipStream_t st = (hipStream_t)stream;
    memcpy(p, ck, nk);
    if (int rc = check_hip(hipMemcpyAsync(d, p, nk, hipMemcpyHostToDevice, st), "hipMemcpyAsync(ck)")) return drained(rc, st);
    if (int rc = launch_encode((const int8_t*)d, (int8_t*)(d + o_dn), B, bgn, Zc, zi, K, N, st)) return drained(rc, st);
    if (int rc = check_hip(hipMemcpyAsync(p + o_dn, d + o_dn, (size_t)B * N, hipMemcpyDeviceToHost, st), "hipMemcpyAsync(dn)"))
        return drained(rc, st);
    if (int rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize")) return rc;
    memcpy(dn, p + o_dn, (size_t)B * N);
    return LDPC5G_OK;
}

int ldpc5g_decode_bf(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L, int32_t flags,
                     int64_t ldl, int64_t ldc, void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    const int N = (bgn == 1 ? 66 : 50) * Zc + (2 - pc) * Zc, Nf = (bgn == 1 ? 68 : 52) * Zc;
    if (B < 0 || L < 0 || (B > 1 && (ldl < N || ldc < Nf)))
        return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d ldl=%lld ldc=%lld (N=%d Nf=%d)", B, L, (long long)ldl, (long long)ldc, N, Nf);
    if (llr_dtype != LDPC5G_F64 && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "bad llr dtype %d", llr_dtype);
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    return launch_bf(bgn, llr_dtype, llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, pc,
                     (hipStream_t)stream);
}

int64_t ldpc5g_bp_scratch_elems(int32_t B, int32_t bgn, int32_t Zc) {
    if ((bgn != 1 && bgn != 2) || B < 0 || zc_index(Zc) < 0) return -1;
    return (int64_t)B * bp_scratch_per_zc(bgn) * Zc;
}

int ldpc5g_decode_bp(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                     double* scratch, int64_t scratch_elems, int32_t B, int32_t bgn, int32_t Zc,
                     int32_t L, int32_t flags, int64_t ldl, int64_t ldc, void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    const int N = (bgn == 1 ? 66 : 50) * Zc + (2 - pc) * Zc, Nf = (bgn == 1 ? 68 : 52) * Zc;
    if (B < 0 || L < 0 || (B > 1 && (ldl < N || ldc < Nf)))
        return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d ldl=%lld ldc=%lld (N=%d Nf=%d)", B, L, (long long)ldl, (long long)ldc, N, Nf);
    if (scratch_elems < ldpc5g_bp_scratch_elems(B, bgn, Zc))
        return fail(LDPC5G_ESIZE, "scratch too small: %lld < %lld", (long long)scratch_elems, (long long)ldpc5g_bp_scratch_elems(B, bgn, Zc));
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters || !scratch) return fail(LDPC5G_ESIZE, "null buffer");
    return launch_bp(bgn, llr, ck, status, iters, scratch, B, Zc, zi, ldl, ldc, L, pc,
                     (hipStream_t)stream);
}

int ldpc5g_decode_ms_mixed(const ldpc5g_cb_desc_t* desc, int32_t B, const void* llr_base,
                           int32_t llr_dtype, int8_t* ck_base, uint8_t* status, int32_t* iters,
                           int32_t L, double alpha, double beta, int32_t schedule, int32_t flags,
                           void* stream) {
    g_err.clear();
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    if (int rc = check_mixed_args(B, L, llr_dtype, schedule, beta)) return rc;
    if (B == 0) return LDPC5G_OK;
    if (!desc || !llr_base || !ck_base || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    const int64_t need = build_plan(desc, B, schedule, nullptr, 0);
    if (need < 0) return (int)need;
    std::vector<unsigned char> host(need);
    build_plan(desc, B, schedule, host.data(), need);
    MixedPlanHdr h;
    memcpy(&h, host.data(), sizeof h);
    hipStream_t st = (hipStream_t)stream;
    // stream-ordered scratch: allocated, filled (from a pinned staging slot), used and freed in
    // stream order
    void* dev = nullptr;
    if (int rc = check_hip(hipMallocAsync(&dev, need, st), "hipMallocAsync(work list)")) return rc;
    int rc = stage_h2d(dev, host.data(), need, st);
    if (!rc) rc = launch_plan(h, (const unsigned char*)dev, llr_base, llr_dtype, ck_base, status, iters, L, alpha, beta, pc,
                              (flags & LDPC5G_RATE_MATCHED) != 0, st);
    const int rc2 = check_hip(hipFreeAsync(dev, st), "hipFreeAsync(work list)");
    return rc ? rc : rc2;
}

int64_t ldpc5g_mixed_plan(const ldpc5g_cb_desc_t* desc, int32_t B, int32_t schedule, void* plan,
                          int64_t plan_bytes) {
    g_err.clear();
    if (B < 0) return fail(LDPC5G_ESIZE, "B=%d", B);
    if (schedule != LDPC5G_FLOODING && schedule != LDPC5G_LAYERED) return fail(LDPC5G_ESIZE, "bad schedule %d", schedule);
    if (B > 0 && !desc) return fail(LDPC5G_ESIZE, "null desc");
    return build_plan(desc, B, schedule, plan, plan_bytes);
}

int ldpc5g_decode_ms_mixed_plan(const void* plan_dev, const void* plan_host, const void* llr_base,
                                int32_t llr_dtype, int8_t* ck_base, uint8_t* status,
                                int32_t* iters, int32_t L, double alpha, double beta,
                                int32_t schedule, int32_t flags, void* stream) {
    g_err.clear();
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    if (!plan_host || !plan_dev) return fail(LDPC5G_ESIZE, "null plan");
    MixedPlanHdr h;
    memcpy(&h, plan_host, sizeof h);
    if (h.magic != kPlanMagic) return fail(LDPC5G_ESIZE, "not a mixed plan (ldpc5g_mixed_plan)");
    if (h.schedule != schedule) return fail(LDPC5G_ESIZE, "plan built for schedule %d, called with %d", h.schedule, schedule);
    if (int rc = check_mixed_args(h.nref, L, llr_dtype, schedule, beta)) return rc;
    if (h.nref == 0) return LDPC5G_OK;
    if (!llr_base || !ck_base || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    return launch_plan(h, (const unsigned char*)plan_dev, llr_base, llr_dtype, ck_base, status, iters, L, alpha, beta, pc,
                       (flags & LDPC5G_RATE_MATCHED) != 0,
                       (hipStream_t)stream);
}

int64_t ldpc5g_sparse_scratch_bytes(int32_t B, int32_t M, int32_t N, int32_t E, int32_t algo) {
    if (B < 0 || M < 0 || N < 1 || E < 0 || algo < LDPC5G_ALGO_MS || algo > LDPC5G_ALGO_BF) return -1;
    if (sparse_lds_bytes(M, N, E, algo)) return 0;
    return (int64_t)B * sparse_cb_bytes(M, N, E, algo);
}

int ldpc5g_decode_sparse(const double* llr, int64_t ldl, int32_t B, int32_t M, int32_t N, int32_t E,
                         const int32_t* row_ptr, const int32_t* col_idx, const int32_t* col_ptr,
                         const int32_t* col_edge, const int32_t* col_row, int32_t L, int32_t algo,
                         double alpha, double beta, int8_t* ck, int64_t ldc, uint8_t* status,
                         int32_t* iters, void* scratch, int64_t scratch_bytes, void* stream) {
    g_err.clear();
    if (algo < LDPC5G_ALGO_MS || algo > LDPC5G_ALGO_BF) return fail(LDPC5G_ESIZE, "bad algo %d", algo);
    if (B < 0 || M < 0 || N < 1 || E < 0 || L < 0 || (B > 1 && (ldl < N || ldc < N)))
        return fail(LDPC5G_ESIZE, "bad sizes B=%d M=%d N=%d E=%d L=%d ldl=%lld ldc=%lld", B, M, N, E, L,
                    (long long)ldl, (long long)ldc);
    const int64_t need = ldpc5g_sparse_scratch_bytes(B, M, N, E, algo);
    if (scratch_bytes < need)
        return fail(LDPC5G_ESIZE, "scratch too small: %lld < %lld", (long long)scratch_bytes, (long long)need);
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters || !row_ptr || !col_ptr || (need > 0 && !scratch) ||
        (E > 0 && (!col_idx || !col_edge || !col_row)))
        return fail(LDPC5G_ESIZE, "null buffer");
    SparseH h{row_ptr, col_idx, col_ptr, col_edge, col_row, M, N, E, 0};
    return launch_sparse(llr, ldl, h, ck, ldc, status, iters, scratch, B, L, algo, alpha, beta,
                         (hipStream_t)stream);
}

}  // extern "C"
