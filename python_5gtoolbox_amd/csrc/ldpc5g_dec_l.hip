// ldpc5g_dec_l.hip — layered float32 min-sum decoder instantiations; built without
// the SLP vectorizer (build.py NO_SLP).  Part of libldpc5g.so (MI355X, gfx950).
#include "ldpc5g_dec_body.h"

namespace ldpc5g_impl {

int dec_blocks_per_cu_l(int bgn) {
    return bgn == 1 ? blocks_per_cu_t<1, float, true>() : blocks_per_cu_t<2, float, true>();
}

int launch_dec_l(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                 int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                 hipStream_t st) {
    return bgn == 1 ? launch_dec_t<1, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_dec_t<2, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_dec_mixed_l(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters,
                       int nwg, const DecWork* work, const CbRef* cbs, int L, double alpha,
                       double beta, int pc, hipStream_t st, bool zc384) {
    if (zc384 && bgn == 1)
        return launch_dec_mixed_t<1, float, true, false, 384>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
    return bgn == 1 ? launch_dec_mixed_t<1, float, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                    : launch_dec_mixed_t<2, float, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
