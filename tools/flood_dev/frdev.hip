// Development harness (not product): the float64 BG1 frame kernel (ldpc5g_dec_frame.h) alone, from
// a (possibly patched) copy of csrc/, for timing beside the product library (tools/flood_dev/run_dev.py).
#include <stdarg.h>
#include <stdio.h>

#include "ldpc5g_dec_frame.h"

#ifndef FRDEV_DEAD
#define FRDEV_DEAD false   // true: the LDPC5G_RATE_MATCHED instantiation
#endif

namespace ldpc5g_impl {
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
    return code;
}
int check_hip(hipError_t e, const char* what) {
    return e == hipSuccess ? 0 : fail(LDPC5G_EHIP, "%s: %s", what, hipGetErrorString(e));
}
}  // namespace ldpc5g_impl

extern "C" int fdev_decode(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                           long long ldl, long long ldc, int L, double alpha, hipStream_t st) {
    using namespace ldpc5g_impl;
    if (Zc != kFrZ) return LDPC5G_EZC;
    constexpr size_t lds = (size_t)kFrPlan<1>.bytes;
    if (int rc = set_lds_once<ldpc_frame_kernel<1, false, FRDEV_DEAD>>(lds)) return rc;
    auto kern = ldpc_frame_kernel<1, false, FRDEV_DEAD>;
    hipLaunchKernelGGL(kern, dim3(B), dim3(kFrThreads), lds, st, llr, ck, status, iters,
                       (int64_t)ldl, (int64_t)ldc, L, alpha, 0.0, 2, (const DecWork*)nullptr, (const CbRef*)nullptr);
    return check_hip(hipGetLastError(), "ldpc_frame_kernel launch");
}
