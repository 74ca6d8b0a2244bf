// ldpc5g_dec_dead_f32.hip — float32 instantiations of the flooding decoder's dead-extension-row
// variants (see ldpc5g_dec_dead.hip); own translation unit.
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {

int launch_flood_dead_f32(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                          int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                          hipStream_t st) {
    return bgn == 1 ? launch_flood_t<1, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_flood_t<2, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_flood_mixed_dead_f32(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                                const DecWork* work, const CbRef* cbs, int L, double alpha, double beta, int pc,
                                hipStream_t st) {
    return bgn == 1 ? launch_flood_mixed_t<1, float, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                    : launch_flood_mixed_t<2, float, true>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
