// ldpc5g_dec_f32.hip — float32 instantiations of the flooding min-sum decoder (batch and mixed work
// lists); own translation unit so it compiles in parallel with the float64 ones (ldpc5g_dec.hip).
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {

int flood_blocks_per_cu_f32(int bgn) {
    return bgn == 1 ? flood_blocks_per_cu_t<1, float>() : flood_blocks_per_cu_t<2, float>();
}

int launch_flood_f32(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                     int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    return bgn == 1 ? launch_flood_t<1, float>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_flood_t<2, float>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int launch_flood_mixed_f32(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                           const DecWork* work, const CbRef* cbs, int L, double alpha, double beta, int pc,
                           hipStream_t st) {
    return bgn == 1 ? launch_flood_mixed_t<1, float>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st)
                    : launch_flood_mixed_t<2, float>(p, ck, status, iters, nwg, work, cbs, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
