// ldpc5g_dec.hip — flooding min-sum decoder instantiations (float64: the drop-in's bit-exact path;
// float32 in ldpc5g_dec_f32.hip) and the decoder dispatch; the layered kernels live in ldpc5g_dec_l.hip.
// Part of libldpc5g.so (MI355X, gfx950).
#include "ldpc5g_dec_flood.h"


namespace ldpc5g_impl {

int dec_blocks_per_cu(int bgn, int dtype, bool layered) {
    if (layered) return dec_blocks_per_cu_l(bgn);
    if (dtype == LDPC5G_F64) return bgn == 1 ? flood_blocks_per_cu_t<1, double>() : flood_blocks_per_cu_t<2, double>();
    return flood_blocks_per_cu_f32(bgn);
}

int launch_dec(int bgn, int dtype, bool layered, const void* llr, int8_t* ck, uint8_t* status,
               int32_t* iters, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L,
               double alpha, double beta, int pc, bool dead, hipStream_t st) {
    if (layered)
        return dead ? launch_dec_l_dead(bgn, (const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_dec_l(bgn, (const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    // a few large float64 codeblocks (the per-codeblock drop-ins): each over several CUs
    // (never while the stream is being captured: the split path may allocate on first use)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (dtype == LDPC5G_F64 && split_wanted(bgn, B, Zc) &&
        (hipStreamIsCapturing(st, &cap) != hipSuccess || cap == hipStreamCaptureStatusNone))
        return launch_flood_split(bgn, (const double*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    // launches whose codeblocks fit 64 slots (one small codeblock per drop-in call): 16 parts
    const int G = std::min(dec_G(Zc, false), B);
    if (G * Zc <= kFloodSmallCS)
        return launch_flood_small(bgn, dtype, llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st);
    if (dead) return launch_flood_dead(bgn, dtype, llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    if (dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        if (LDPC5G_FLOOD_FRAME && Zc == kFrameZc)
            return launch_frame(bgn, false, p, ck, status, iters, B, ldl, ldc, L, alpha, beta, pc, nullptr, nullptr, st);
        return bgn == 1 ? launch_flood_t<1, double>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                        : launch_flood_t<2, double>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    }
    return launch_flood_f32(bgn, (const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_dec_mixed(int bgn, int dtype, bool layered, const void* llr, int8_t* ck,
                     uint8_t* status, int32_t* iters, int nwg, const DecWork* work,
                     const CbRef* cbs, int L, double alpha, double beta, int pc, bool dead,
                     hipStream_t st, bool zc384) {
    if (layered)
        return dead ? launch_dec_mixed_l_dead(bgn, (const float*)llr, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st, zc384)
                    : launch_dec_mixed_l(bgn, (const float*)llr, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st, zc384);
    if (dead) return launch_flood_mixed_dead(bgn, dtype, llr, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st, zc384);
    if (dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        if (zc384 && LDPC5G_FLOOD_FRAME)
            return launch_frame(bgn, false, p, ck, status, iters, nwg, 0, 0, L, alpha, beta, pc, work, cbs, st);
        if constexpr (!LDPC5G_FLOOD_FRAME)
            if (zc384 && bgn == 1)
                return launch_flood_mixed_t<1, double, false, 384>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
        return bgn == 1 ? launch_flood_mixed_t<1, double>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                        : launch_flood_mixed_t<2, double>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
    }
    return launch_flood_mixed_f32(bgn, (const float*)llr, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
