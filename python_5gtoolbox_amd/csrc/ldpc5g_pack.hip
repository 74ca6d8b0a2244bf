// ldpc5g_pack.hip — gather records for the multi-GPU path.  A record is one row
// of bytes: the row's bits (int8 0/1, the reference's one-bit-per-byte layout) packed in
// np.packbits order (bit i -> byte i/8, bit 7 - i%8), then optionally a status byte and a
// little-endian int32 (iterations).  A rank's decoded shard (4096 BG1 Zc=384 codeblocks: 34.6 MB
// of info bytes) becomes 4096 x 1061 B = 4.3 MB, one contiguous block, so the gather to rank 0 is
// a single RCCL collective of 1/8 the bytes.  HBM-bound, one pass each way.
#include <stdint.h>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {

// one thread per packed byte of row blockIdx.y (8 input bytes as two words when the row is
// 4-byte aligned); thread 0 of the row also writes the tail fields
__global__ __launch_bounds__(256) void pack_records_kernel(const int8_t* __restrict__ bits, int64_t ldb,
                                                           int64_t nbits, const uint8_t* __restrict__ status,
                                                           const int32_t* __restrict__ iters,
                                                           uint8_t* __restrict__ rec, int64_t ldr,
                                                           bool aligned) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nbytes = (nbits + 7) >> 3;
    const int64_t r = blockIdx.y;
    uint8_t* row = rec + r * ldr;
    if (j == 0) {
        int64_t o = nbytes;
        if (status) row[o++] = status[r];
        if (iters) {
            const uint32_t v = (uint32_t)iters[r];
#pragma unroll
            for (int b = 0; b < 4; ++b) row[o + b] = (uint8_t)(v >> (8 * b));
        }
    }
    if (j >= nbytes) return;
    const int8_t* src = bits + r * ldb + 8 * j;
    uint32_t v = 0;
    if (aligned && 8 * j + 8 <= nbits) {
        const uint64_t w = ((uint64_t)(*(const uint32_t*)(src + 4)) << 32) | *(const uint32_t*)src;
#pragma unroll
        for (int i = 0; i < 8; ++i) v |= (uint32_t)((w >> (8 * i)) & 1u) << (7 - i);
    } else {
        for (int i = 0; i < 8 && 8 * j + i < nbits; ++i) v |= (uint32_t)(src[i] & 1) << (7 - i);
    }
    row[j] = (uint8_t)v;
}

// one thread per packed byte: its 8 bits become one 8-byte store when the output row is
// 8-byte aligned, byte stores otherwise (and in the tail byte)
__global__ __launch_bounds__(256) void unpack_records_kernel(const uint8_t* __restrict__ rec, int64_t ldr,
                                                             int64_t nbits, int8_t* __restrict__ bits,
                                                             int64_t ldb, uint8_t* __restrict__ status,
                                                             int32_t* __restrict__ iters, int64_t fs,
                                                             bool aligned) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = blockIdx.y;
    const int64_t nbytes = (nbits + 7) >> 3;
    const uint8_t* row = rec + r * ldr;
    if (j == 0) {
        int64_t o = nbytes;
        if (status) status[r * fs] = row[o++];
        if (iters) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) v |= (uint32_t)row[o + b] << (8 * b);
            iters[r * fs] = (int32_t)v;
        }
    }
    if (!bits || j >= nbytes) return;
    const uint32_t v = row[j];
    int8_t* dst = bits + r * ldb + 8 * j;
    if (aligned && 8 * j + 8 <= nbits) {
        uint64_t w = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) w |= (uint64_t)((v >> (7 - i)) & 1u) << (8 * i);
        *(uint64_t*)dst = w;
    } else {
        for (int i = 0; i < 8 && 8 * j + i < nbits; ++i) dst[i] = (int8_t)((v >> (7 - i)) & 1u);
    }
}

int64_t rec_bytes(int64_t nbits, bool st, bool it) { return (nbits + 7) / 8 + (st ? 1 : 0) + (it ? 4 : 0); }

}  // namespace
}  // namespace ldpc5g_impl

using namespace ldpc5g_impl;

extern "C" {

int ldpc5g_pack_records(const int8_t* bits, int64_t ldb, int32_t R, int64_t nbits,
                        const uint8_t* status, const int32_t* iters, uint8_t* rec, int64_t ldr,
                        void* stream) {
    clear_error();
    const int64_t need = rec_bytes(nbits, status != nullptr, iters != nullptr);
    if (R < 0 || R > 65535 || nbits < 0 || (R > 1 && (ldb < nbits || ldr < need)) || (R == 1 && ldr < need && ldr != 0))
        return fail(LDPC5G_ESIZE, "bad sizes R=%d nbits=%lld ldb=%lld ldr=%lld (record %lld B)", R, (long long)nbits, (long long)ldb, (long long)ldr, (long long)need);
    if (R == 0 || need == 0) return LDPC5G_OK;
    if (!rec || (nbits && !bits)) return fail(LDPC5G_ESIZE, "null buffer");
    const int64_t nbytes = (nbits + 7) / 8;
    const bool aligned = ((uintptr_t)bits & 3) == 0 && (ldb & 3) == 0;
    hipLaunchKernelGGL(pack_records_kernel, dim3((unsigned)((nbytes + 255) / 256 + (nbytes == 0)), R), dim3(256), 0,
                       (hipStream_t)stream, bits, ldb, nbits, status, iters, rec, ldr, aligned);
    return check_hip(hipGetLastError(), "pack_records launch");
}

int ldpc5g_unpack_records(const uint8_t* rec, int64_t ldr, int32_t R, int64_t nbits, int8_t* bits,
                          int64_t ldb, uint8_t* status, int32_t* iters, int64_t fstride,
                          void* stream) {
    clear_error();
    const int64_t need = rec_bytes(nbits, status != nullptr, iters != nullptr);
    if (R < 0 || R > 65535 || nbits < 0 || (R > 1 && ((bits && ldb < nbits) || ldr < need)))
        return fail(LDPC5G_ESIZE, "bad sizes R=%d nbits=%lld ldb=%lld ldr=%lld (record %lld B)", R, (long long)nbits, (long long)ldb, (long long)ldr, (long long)need);
    if (R == 0 || need == 0) return LDPC5G_OK;
    if (!rec) return fail(LDPC5G_ESIZE, "null buffer");
    if (fstride < 1) return fail(LDPC5G_ESIZE, "fstride=%lld", (long long)fstride);
    const int64_t nbytes = (nbits + 7) / 8;
    const bool aligned = ((uintptr_t)bits & 7) == 0 && (ldb & 7) == 0;
    hipLaunchKernelGGL(unpack_records_kernel, dim3((unsigned)((nbytes + 255) / 256 + (nbytes == 0)), R), dim3(256), 0,
                       (hipStream_t)stream, rec, ldr, nbits, bits, ldb, status, iters, fstride, aligned);
    return check_hip(hipGetLastError(), "unpack_records launch");
}

}  // extern "C"
