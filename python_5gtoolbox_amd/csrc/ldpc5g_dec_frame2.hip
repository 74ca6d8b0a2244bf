// ldpc5g_dec_frame2.hip — the float64 Zc = 384 frame kernel (ldpc5g_dec_frame.h) for base graph 2: its own
// translation unit (the four compile in parallel); declared in ldpc5g_common.h.
#include "ldpc5g_dec_frame.h"

namespace ldpc5g_impl {

template <int BG, bool DEAD>
int launch_frame_bg(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg, int64_t ldl,
                    int64_t ldc, int L, double alpha, double beta, int pc, const DecWork* work,
                    const CbRef* cbs, hipStream_t st) {
    return launch_frame_t<BG, DEAD>(llr, ck, status, iters, nwg, ldl, ldc, L, alpha, beta, pc, work, cbs, st);
}
template int launch_frame_bg<2, false>(const double*, int8_t*, uint8_t*, int32_t*, int, int64_t, int64_t, int,
                                    double, double, int, const DecWork*, const CbRef*, hipStream_t);

}  // namespace ldpc5g_impl
