// ldpc5g_dec_flood16.hip — the flooding decoder's small launches (codeblocks of at most 64 slots,
// e.g. ONE BG2 Zc=8 codeblock per call from the per-codeblock drop-ins, BASELINE config 1): the
// small-codeblock kernel (ldpc5g_dec_small.h: a thread per check node, two barriers per iteration)
// where its LDS fits, else the batch kernel's 16 parts x 64 slots (1024 threads) configuration.  float64 here, float32 in ldpc5g_dec_flood16_f32.hip
// (own translation units: they compile in parallel).
#include "ldpc5g_dec_small.h"

namespace ldpc5g_impl {

int launch_flood_small(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                       int B, int Zc, int zi, int G, int64_t ldl, int64_t ldc, int L, double alpha,
                       double beta, int pc, hipStream_t st) {
    constexpr int NP = kFloodSmallNP, CS = kFloodSmallCS;
    if (dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        // a thread per check node, two barriers per iteration (ldpc5g_dec_small.h)
        if (bgn == 1 ? small_fits<1, double>(Zc) : small_fits<2, double>(Zc))
            return bgn == 1 ? launch_small_t<1, double>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                            : launch_small_t<2, double>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
        return bgn == 1 ? launch_flood_cfg<1, double, NP, CS>(p, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st)
                        : launch_flood_cfg<2, double, NP, CS>(p, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st);
    }
    return launch_flood_small_f32(bgn, (const float*)llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta,
                                  pc, st);
}

}  // namespace ldpc5g_impl
