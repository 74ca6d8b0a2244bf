// Development harness (not product): the small-codeblock decoder (ldpc5g_dec_small.h) compiled on
// its own, optionally with phase timestamps (-DLDPC5G_SMALL_TS: thread 0 records s_memtime at the
// phase boundaries of the first iterations into the first bytes of its ck row), for timing variants
// beside the product library (tools/small_dev/run_sdev.py).
#include <stdarg.h>
#include <stdio.h>

#include "ldpc5g_dec_small.h"

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

extern "C" int sdev_decode(int bg, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                           long long ldl, long long ldc, int L, double alpha, hipStream_t st) {
    using namespace ldpc5g_impl;
    int zi = -1;
    for (int i = 0; i < LDPC5G_NUM_ZC; ++i)
        if (kLdpcZcList[i] == Zc) zi = i;
    if (zi < 0) return LDPC5G_EZC;
    return bg == 1 ? launch_small_t<1, double>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, 0.0, 2, st)
                   : launch_small_t<2, double>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, 0.0, 2, st);
}
