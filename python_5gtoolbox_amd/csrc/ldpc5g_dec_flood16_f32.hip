// ldpc5g_dec_flood16_f32.hip — float32 instantiations of the flooding decoder's small-launch
// configuration (16 parts x 64 slots, see ldpc5g_dec_flood16.hip); own translation unit.
#include "ldpc5g_dec_small.h"

namespace ldpc5g_impl {

int launch_flood_small_f32(int bgn, const float* p, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                           int zi, int G, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                           hipStream_t st) {
    constexpr int NP = kFloodSmallNP, CS = kFloodSmallCS;
    if (bgn == 1 ? small_fits<1, float>(Zc) : small_fits<2, float>(Zc))
        return bgn == 1 ? launch_small_t<1, float>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                        : launch_small_t<2, float>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    return bgn == 1 ? launch_flood_cfg<1, float, NP, CS>(p, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st)
                    : launch_flood_cfg<2, float, NP, CS>(p, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st);
}

}  // namespace ldpc5g_impl
