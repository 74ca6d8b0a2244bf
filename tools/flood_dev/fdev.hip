// Development harness (not product): one instantiation of the float64 BG1 flooding kernel from a
// (possibly patched) copy of csrc/, so a variant compiles in about a minute and can be timed
// beside the product library (tools/flood_dev/run_dev.py).
#include <stdarg.h>
#include <stdio.h>

#include "ldpc5g_dec_flood.h"

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
    int zi = -1;
    for (int i = 0; i < LDPC5G_NUM_ZC; ++i)
        if (kLdpcZcList[i] == Zc) zi = i;
    if (zi < 0) return LDPC5G_EZC;
    return launch_flood_t<1, double>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, 0.0, 2, st);
}
