// ldpc5g_dec_l_dead.hip — the layered float32 decoder's dead-extension-row variant (DEAD = true,
// selected by LDPC5G_RATE_MATCHED: rate-recovered LLR rows whose untransmitted parity columns
// are +0.0).  Own translation unit so the headline instantiations
// (ldpc5g_dec_l.hip) compile unchanged and in parallel; built without the SLP vectorizer too.
#include "ldpc5g_dec_body.h"

namespace ldpc5g_impl {

int launch_dec_l_dead(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                      int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta,
                      int pc, hipStream_t st) {
    return bgn == 1 ? launch_dec_t<1, float, true, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_dec_t<2, float, true, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_dec_mixed_l_dead(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters,
                            int nwg, const DecWork* work, const CbRef* cbs, int L, double alpha,
                            double beta, int pc, hipStream_t st, bool zc384) {
    if (zc384 && bgn == 1)
        return launch_dec_mixed_t<1, float, true, true, 384>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
    return bgn == 1 ? launch_dec_mixed_t<1, float, true, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                    : launch_dec_mixed_t<2, float, true, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
