// ldpc5g_dec_dead.hip — the flooding decoder's dead-extension-row variants (DEAD = true, float64
// batch and mixed work lists), selected by LDPC5G_RATE_MATCHED: float64 here,
// float32 in ldpc5g_dec_dead_f32.hip.  Own translation units: they compile in parallel.
#include "ldpc5g_dec_flood.h"


namespace ldpc5g_impl {

int launch_flood_dead(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status,
                      int32_t* iters, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L,
                      double alpha, double beta, int pc, hipStream_t st) {
    if (dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        if (LDPC5G_FLOOD_FRAME && Zc == kFrameZc)
            return launch_frame(bgn, true, p, ck, status, iters, B, ldl, ldc, L, alpha, beta, pc, nullptr, nullptr, st);
        return bgn == 1 ? launch_flood_t<1, double, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                        : launch_flood_t<2, double, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    }
    return launch_flood_dead_f32(bgn, (const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_flood_mixed_dead(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status,
                            int32_t* iters, int nwg, const DecWork* work, const CbRef* cbs, int L,
                            double alpha, double beta, int pc, hipStream_t st, bool zc384) {
    if (dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        if (zc384 && LDPC5G_FLOOD_FRAME)
            return launch_frame(bgn, true, p, ck, status, iters, nwg, 0, 0, L, alpha, beta, pc, work, cbs, st);
        if constexpr (!LDPC5G_FLOOD_FRAME)
            if (zc384 && bgn == 1)
                return launch_flood_mixed_t<1, double, true, 384>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
        return bgn == 1 ? launch_flood_mixed_t<1, double, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                        : launch_flood_mixed_t<2, double, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
    }
    return launch_flood_mixed_dead_f32(bgn, (const float*)llr, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc,
                                       st);
}

}  // namespace ldpc5g_impl
