// ldpc5g_phy.hip — the symbol-level steps either side of the DL-SCH chain,
// on the GPU and batched over transport blocks:
//   Gold-sequence scrambling code c(n) ....... py5gphy/common/nrPRBS.py:5-25 (gen_nrPRBS)
//   scrambling + modulation mapper ........... py5gphy/nr_pdsch/nr_pdsch_process.py:17-25,
//                                              py5gphy/common/nrModulation.py:4-42 (all seven)
//   soft demodulation + descrambling ......... py5gphy/demodulation/nr_Demodulation.py:12-46,
//                                              demod_{bpsk,pi2_bpsk,qpsk,16qam,64qam,256qam,1024qam}.py,
//                                              py5gphy/nr_pdsch/nr_pdsch.py:268-274
// All elementwise / HBM-bound.  The scrambling code is produced 32 bits per word (packed LSB
// first, bit k of word w = c(32w + k)): a thread jumps both m-sequences to its first word with
// constexpr GF(2) matrix powers T^(2^i), then steps 32 positions at a time with shifts.
#include <math.h>
#include <stdint.h>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {

// ============================================================================ Gold sequence
constexpr int kPrbsPow = 26;   // jumps up to 2^26 positions (G + 1600 < 67 M bits)
struct PrbsTables {
    uint32_t t[2][kPrbsPow][31];   // [x1 / x2][i][column j] of T^(2^i), T = one LFSR step
};
// State S(n) of an m-sequence: bit i = x(n + i), i = 0..30.  One step: bit i <- bit i+1,
// bit 30 <- x(n+31) = XOR of the taps (x1: x(n+3) + x(n); x2: x(n+3) + x(n+2) + x(n+1) + x(n)).
__host__ __device__ constexpr uint32_t mat_apply(const uint32_t (&M)[31], uint32_t v) {
    uint32_t r = 0;
    for (int j = 0; j < 31; ++j)
        if ((v >> j) & 1u) r ^= M[j];
    return r;
}
constexpr PrbsTables make_prbs_tables() {
    PrbsTables P{};
    for (int q = 0; q < 2; ++q) {
        const uint32_t taps = q == 0 ? 0x9u : 0xfu;   // x1: {0, 3}; x2: {0, 1, 2, 3}
        for (int j = 0; j < 31; ++j)
            P.t[q][0][j] = (j >= 1 ? 1u << (j - 1) : 0u) | (((taps >> j) & 1u) ? 1u << 30 : 0u);
        for (int i = 1; i < kPrbsPow; ++i)
            for (int j = 0; j < 31; ++j) P.t[q][i][j] = mat_apply(P.t[q][i - 1], P.t[q][i - 1][j]);
    }
    return P;
}
__constant__ PrbsTables kPrbs = make_prbs_tables();

__device__ uint32_t prbs_jump(int q, uint32_t s, uint32_t n) {
    for (int i = 0; i < kPrbsPow; ++i) {
        if ((n >> i) & 1u) {
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 31; ++j) r ^= ((s >> j) & 1u) ? kPrbs.t[q][i][j] : 0u;
            s = r;
        }
    }
    return s;
}

// x(m .. m+31) of an m-sequence from its state at m; `s` becomes the state at m + 32.
__device__ __forceinline__ uint32_t prbs_step32(uint32_t& s, bool x2) {
    uint64_t W = s;
    const uint64_t n1 = x2 ? (W ^ (W >> 1) ^ (W >> 2) ^ (W >> 3)) : (W ^ (W >> 3));
    W |= (n1 & 0x0FFFFFFFull) << 31;                      // x(m+31 .. m+58)
    const uint64_t n2 = x2 ? ((W >> 28) ^ (W >> 29) ^ (W >> 30) ^ (W >> 31)) : ((W >> 28) ^ (W >> 31));
    W |= (n2 & 0xFull) << 59;                             // x(m+59 .. m+62)
    s = (uint32_t)(W >> 32) & 0x7FFFFFFFu;
    return (uint32_t)W;
}

constexpr int kPrbsWordsPerThread = 8;
constexpr int kPrbsLaneLog = 8;   // log2(32 * kPrbsWordsPerThread): bits per thread
static_assert(32 * kPrbsWordsPerThread == 1 << kPrbsLaneLog, "bits per thread must be 2^kPrbsLaneLog");

// T^(m 2^kPrbsLaneLog) s for m < 256: the per-thread part of the jump
__device__ __forceinline__ uint32_t prbs_jump_lane(int q, uint32_t s, uint32_t m) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if ((m >> i) & 1u) {
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 31; ++j) r ^= ((s >> j) & 1u) ? kPrbs.t[q][kPrbsLaneLog + i][j] : 0u;
            s = r;
        }
    }
    return s;
}

// words[t][w] = c(32w .. 32w+31) of transport block t (gen_nrPRBS(cinit[t], ...) packed).  The
// jump to the workgroup's first bit is uniform (scalar); each thread then jumps by
// threadIdx.x * 256 bits with at most 8 matrix products.
__global__ __launch_bounds__(256) void prbs_kernel(const uint32_t* __restrict__ cinit, int64_t nw,
                                                   uint32_t* __restrict__ words, int64_t ldw) {
    const int t = blockIdx.y;
    const int64_t wb = (int64_t)blockIdx.x * 256 * kPrbsWordsPerThread;
    const int64_t w0 = wb + (int64_t)threadIdx.x * kPrbsWordsPerThread;
    const uint32_t nb = 1600u + 32u * (uint32_t)wb;
    uint32_t s1 = prbs_jump(0, 1u, nb);
    uint32_t s2 = prbs_jump(1, cinit[t] & 0x7FFFFFFFu, nb);
    if (w0 >= nw) return;
    s1 = prbs_jump_lane(0, s1, threadIdx.x);
    s2 = prbs_jump_lane(1, s2, threadIdx.x);
    uint32_t* out = words + (int64_t)t * ldw;
#pragma unroll
    for (int k = 0; k < kPrbsWordsPerThread; ++k) {
        const uint32_t c = prbs_step32(s1, false) ^ prbs_step32(s2, true);
        if (w0 + k < nw) out[w0 + k] = c;
    }
}

__device__ __forceinline__ uint32_t prbs_bits(const uint32_t* w, int64_t pos, int n) {   // n <= 8
    const int64_t q = pos >> 5;
    const int sh = (int)(pos & 31);
    uint32_t v = w[q] >> sh;
    if (sh + n > 32) v |= w[q + 1] << (32 - sh);
    return v & ((1u << n) - 1u);
}

// ======================================================================== modulation mapper
// scrambled bit b'(i) = b(i) + c(i) mod 2; symbol = (level_re + j level_im) / sqrt(scale) in the
// reference's float32 arithmetic: levels exact, then numpy's complex64 division by a real scalar,
// i.e. a multiply by the float32 reciprocal scl = 1 / float32(sqrt(scale)).
// QM = 1: BPSK (re = im = 1 - 2b, nrModulation.py:15-16); with PI2, odd symbols re = 2b - 1
// (pi/2-BPSK, :17-21).  QM = 10: 1024QAM (:38-42).
template <int QM, bool PI2>
__global__ __launch_bounds__(256) void scramble_modulate_kernel(const int8_t* __restrict__ bits,
                                                                int64_t ldb,
                                                                const uint32_t* __restrict__ prbs,
                                                                int64_t ldw, int64_t nsym,
                                                                float scl, float2* __restrict__ sym,
                                                                int64_t ldsym) {
    const int t = blockIdx.y;
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nsym) return;
    const int8_t* b = bits + (int64_t)t * ldb + m * QM;
    uint32_t c = prbs ? prbs_bits(prbs + (int64_t)t * ldw, m * QM, QM) : 0u;
    float u[QM];
#pragma unroll
    for (int i = 0; i < QM; ++i) u[i] = 1.0f - 2.0f * (float)(((uint32_t)b[i] ^ (c >> i)) & 1u);
    float re, im;
    if constexpr (QM == 1) {
        re = (PI2 && (m & 1)) ? -u[0] : u[0], im = u[0];
    } else if constexpr (QM == 2) {
        re = u[0], im = u[1];
    } else if constexpr (QM == 4) {
        re = u[0] * (2.0f - u[2]), im = u[1] * (2.0f - u[3]);
    } else if constexpr (QM == 6) {
        re = u[0] * (4.0f - u[2] * (2.0f - u[4]));
        im = u[1] * (4.0f - u[3] * (2.0f - u[5]));
    } else if constexpr (QM == 8) {
        re = u[0] * (8.0f - u[2] * (4.0f - u[4] * (2.0f - u[6])));
        im = u[1] * (8.0f - u[3] * (4.0f - u[5] * (2.0f - u[7])));
    } else {
        re = u[0] * (16.0f - u[2] * (8.0f - u[4] * (4.0f - u[6] * (2.0f - u[8]))));
        im = u[1] * (16.0f - u[3] * (8.0f - u[5] * (4.0f - u[7] * (2.0f - u[9]))));
    }
    sym[(int64_t)t * ldsym + m] = make_float2(re * scl, im * scl);
}

// ===================================================================== soft demodulation
// Piecewise-linear max-log segments of the reference's demod_*.py, per PAM bit pair p (bits 2p /
// 2p+1 from the real / imaginary part): r < thr*A  ->  LLR = (k*A) * (s*r + (s*c)*A) / nv, or
// (k*A) * r / nv when c = 0.  The 1024QAM table is extracted from demod_1024qam.py by
// tools/gen_demod_tables.py (its if/elif chains, verbatim coefficients).
struct Seg {
    int8_t thr, k, s, c;   // thr = 127: +inf
};
constexpr int kSegMax = 31;
struct SegTable {
    int8_t nseg[5];
    Seg seg[5][kSegMax];
};
constexpr SegTable kSegQpsk = {{1}, {{{127, 4, 1, 0}}}};
constexpr SegTable kSeg16 = {{3, 2},
                             {{{-2, 8, 1, 1}, {2, 4, 1, 0}, {127, 8, 1, -1}},
                              {{0, 4, 1, 2}, {127, 4, -1, -2}}}};
constexpr SegTable kSeg64 = {{7, 6, 4},
                             {{{-6, 16, 1, 3}, {-4, 12, 1, 2}, {-2, 8, 1, 1}, {2, 4, 1, 0}, {4, 8, 1, -1}, {6, 12, 1, -2}, {127, 16, 1, -3}},
                              {{-6, 8, 1, 5}, {-2, 4, 1, 4}, {0, 8, 1, 3}, {2, 8, -1, -3}, {6, 4, -1, -4}, {127, 8, -1, -5}},
                              {{-4, 4, 1, 6}, {0, 4, -1, 2}, {4, 4, 1, -2}, {127, 4, -1, -6}}}};
constexpr SegTable kSeg256 = {{15, 14, 12, 8},
                              {{{-14, 32, 1, 7}, {-12, 28, 1, 6}, {-10, 24, 1, 5}, {-8, 20, 1, 4}, {-6, 16, 1, 3}, {-4, 12, 1, 2}, {-2, 8, 1, 1}, {2, 4, 1, 0},
                                {4, 8, 1, -1}, {6, 12, 1, -2}, {8, 16, 1, -3}, {10, 20, 1, -4}, {12, 24, 1, -5}, {14, 28, 1, -6}, {127, 32, 1, -7}},
                               {{-14, 16, 1, 11}, {-12, 12, 1, 10}, {-10, 8, 1, 9}, {-6, 4, 1, 8}, {-4, 8, 1, 7}, {-2, 12, 1, 6}, {0, 16, 1, 5},
                                {2, 16, -1, -5}, {4, 12, -1, -6}, {6, 8, -1, -7}, {10, 4, -1, -8}, {12, 8, -1, -9}, {14, 12, -1, -10}, {127, 16, -1, -11}},
                               {{-14, 8, 1, 13}, {-10, 4, 1, 12}, {-8, 8, 1, 11}, {-6, 8, -1, 5}, {-2, 4, -1, 4}, {0, 8, -1, 3}, {2, 8, 1, -3},
                                {6, 4, 1, -4}, {8, 8, 1, -5}, {10, 8, -1, -11}, {14, 4, -1, -12}, {127, 8, -1, -13}},
                               {{-12, 4, 1, 14}, {-8, 4, -1, 10}, {-4, 4, 1, 6}, {0, 4, -1, 2}, {4, 4, 1, -2}, {8, 4, -1, -6}, {12, 4, 1, -10},
                                {127, 4, -1, -14}}}};
#include "ldpc5g_demod1024.h"
template <int QM>
constexpr const SegTable& seg_table() {
    if constexpr (QM == 2) return kSegQpsk;
    else if constexpr (QM == 4) return kSeg16;
    else if constexpr (QM == 6) return kSeg64;
    else if constexpr (QM == 8) return kSeg256;
    else return kSeg1024;
}

// One LLR in the arithmetic type C of the input symbols: double for complex128; float for
// complex64, where numpy >= 2 evaluates demod_*.py's scalar expressions in float32 with every
// Python-float constant (k*A, c*A, thr*A) rounded to float32 first (NEP 50) — comparisons too.
template <int QM, int P, typename C>
__device__ __forceinline__ C demod_llr(C r, double A, C nv) {
    constexpr const SegTable& T = seg_table<QM>();
    constexpr int n = T.nseg[P];
    // the reference's if / elif chain: the first segment with r < thr * A; scanned from the top
    // so the lowest matching segment is selected last (all selects, no branches)
    constexpr Seg top = T.seg[P][n - 1];
    C kA = (C)((double)top.k * A), sr = (C)top.s, cA = (C)((double)(top.s * top.c) * A);
    bool noc = top.c == 0;
    sfor<0, n - 1>([&](auto ic) {
        constexpr int i = n - 2 - decltype(ic)::value;
        constexpr Seg g = T.seg[P][i];
        const bool hit = r < (C)((double)g.thr * A);
        kA = hit ? (C)((double)g.k * A) : kA;
        sr = hit ? (C)g.s : sr;
        cA = hit ? (C)((double)(g.s * g.c) * A) : cA;
        noc = hit ? (g.c == 0) : noc;
    });
    const C x = noc ? r : sr * r + cA;
    return (kA * x) / nv;
}

template <typename T>
__device__ __forceinline__ T flip_sign(T v, uint32_t bit) {
    if constexpr (sizeof(T) == 4) return __uint_as_float(__float_as_uint(v) ^ (bit << 31));
    else return __longlong_as_double(__double_as_longlong(v) ^ ((long long)bit << 63));
}

// QM = 1: BPSK LLR = 4 (re + im) A / nv (demod_bpsk.py:9); with PI2, odd symbols use
// 4 (-re + im) A / nv (demod_pi2_bpsk.py:11-12).  Tout = double only for BPSK on complex128
// input, whose reference result stays float64 (no float32 store in demod_bpsk.py).
template <int QM, bool PI2, typename Tin, typename Tout>
__global__ __launch_bounds__(256) void demod_descramble_kernel(const Tin* __restrict__ sym,
                                                               int64_t ldsym,
                                                               const float* __restrict__ nvar,
                                                               int64_t ldnv,
                                                               const uint32_t* __restrict__ prbs,
                                                               int64_t ldw, int64_t nsym, double A,
                                                               Tout* __restrict__ llr,
                                                               int64_t ldllr) {
    using C = decltype(Tin{}.x);
    const int t = blockIdx.y;
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nsym) return;
    const Tin y = sym[(int64_t)t * ldsym + m];
    const C re = y.x, im = y.y;
    const C nv = (C)nvar[(int64_t)t * ldnv + m];
    const uint32_t c = prbs ? prbs_bits(prbs + (int64_t)t * ldw, m * QM, QM) : 0u;
    Tout v[QM];
    if constexpr (QM == 1) {
        const C sre = (PI2 && (m & 1)) ? -re + im : re + im;
        v[0] = (Tout)(((C)4 * sre) * (C)A / nv);
    } else {
        sfor<0, QM / 2>([&](auto pc) {
            constexpr int p = decltype(pc)::value;
            v[2 * p] = (Tout)demod_llr<QM, p>(re, A, nv);
            v[2 * p + 1] = (Tout)demod_llr<QM, p>(im, A, nv);
        });
    }
    Tout* out = llr + (int64_t)t * ldllr + m * QM;
#pragma unroll
    for (int i = 0; i < QM; ++i)   // descrambling: LLR * (1 - 2c), an exact sign flip
        out[i] = flip_sign(v[i], (c >> i) & 1u);
}

// modulation id -> (Qm, pi/2): LDPC5G_PI2_BPSK = -1, otherwise the order Qm itself
int mod_scale(int Qm) {   // sqrt(scale) of nrModulation.py / A = 1 / sqrt(scale) of demod_*.py
    return Qm == 1 ? 2 : Qm == 2 ? 2 : Qm == 4 ? 10 : Qm == 6 ? 42 : Qm == 8 ? 170 : 682;
}
bool mod_ok(int mod) { return mod == -1 || mod == 1 || mod == 2 || mod == 4 || mod == 6 || mod == 8 || mod == 10; }

}  // namespace
}  // namespace ldpc5g_impl

using namespace ldpc5g_impl;

extern "C" {

int ldpc5g_prbs(const uint32_t* cinit, int32_t T, int64_t nbits, uint32_t* words, int64_t ldw,
                void* stream) {
    clear_error();
    const int64_t nw = (nbits + 31) / 32;
    if (T < 0 || nbits < 0 || (T > 1 && ldw < nw)) return fail(LDPC5G_ESIZE, "bad sizes T=%d nbits=%lld ldw=%lld", T, (long long)nbits, (long long)ldw);
    if (1600 + 32 * (nw + kPrbsWordsPerThread) >= (int64_t(1) << kPrbsPow)) return fail(LDPC5G_ESIZE, "nbits=%lld too long", (long long)nbits);
    if (T == 0 || nw == 0) return LDPC5G_OK;
    if (!cinit || !words) return fail(LDPC5G_ESIZE, "null buffer");
    const int64_t nthr = (nw + kPrbsWordsPerThread - 1) / kPrbsWordsPerThread;
    hipLaunchKernelGGL(prbs_kernel, dim3((unsigned)((nthr + 255) / 256), T), dim3(256), 0,
                       (hipStream_t)stream, cinit, nw, words, ldw);
    return check_hip(hipGetLastError(), "prbs_kernel launch");
}

int ldpc5g_scramble_modulate(const int8_t* bits, int64_t ldb, const uint32_t* prbs, int64_t ldw,
                             int32_t T, int64_t nbits, int32_t mod, void* sym, int64_t ldsym,
                             void* stream) {
    clear_error();
    if (!mod_ok(mod)) return fail(LDPC5G_ESIZE, "modulation %d (1 BPSK, -1 pi/2-BPSK, 2/4/6/8/10 QPSK..1024QAM)", mod);
    const int Qm = mod < 0 ? 1 : mod;
    if (T < 0 || nbits < 0 || nbits % Qm) return fail(LDPC5G_ESIZE, "bad sizes T=%d nbits=%lld", T, (long long)nbits);
    const int64_t nsym = nbits / Qm;
    if (T > 1 && (ldb < nbits || ldsym < nsym || (prbs && ldw < (nbits + 31) / 32))) return fail(LDPC5G_ESIZE, "bad strides");
    if (T == 0 || nsym == 0) return LDPC5G_OK;
    if (!bits || !sym) return fail(LDPC5G_ESIZE, "null buffer");
    const float scl = 1.0f / (float)sqrt((double)mod_scale(Qm));
    const dim3 grid((unsigned)((nsym + 255) / 256), T), blk(256);
    hipStream_t st = (hipStream_t)stream;
    float2* out = (float2*)sym;
#define LDPC5G_MOD(QM, PI2) \
    hipLaunchKernelGGL((scramble_modulate_kernel<QM, PI2>), grid, blk, 0, st, bits, ldb, prbs, ldw, nsym, scl, out, ldsym)
    switch (mod) {
        case -1: LDPC5G_MOD(1, true); break;
        case 1: LDPC5G_MOD(1, false); break;
        case 2: LDPC5G_MOD(2, false); break;
        case 4: LDPC5G_MOD(4, false); break;
        case 6: LDPC5G_MOD(6, false); break;
        case 8: LDPC5G_MOD(8, false); break;
        default: LDPC5G_MOD(10, false); break;
    }
#undef LDPC5G_MOD
    return check_hip(hipGetLastError(), "scramble_modulate launch");
}

int ldpc5g_demod_descramble(const void* sym, int32_t sym_dtype, int64_t ldsym, const float* noise_var,
                            int64_t ldnv, const uint32_t* prbs, int64_t ldw, int32_t T, int64_t nsym,
                            int32_t mod, void* llr, int32_t llr_dtype, int64_t ldllr, void* stream) {
    clear_error();
    if (!mod_ok(mod)) return fail(LDPC5G_ESIZE, "modulation %d (1 BPSK, -1 pi/2-BPSK, 2/4/6/8/10 QPSK..1024QAM)", mod);
    const int Qm = mod < 0 ? 1 : mod;
    if (sym_dtype != LDPC5G_F32 && sym_dtype != LDPC5G_F64) return fail(LDPC5G_ESIZE, "bad symbol dtype %d", sym_dtype);
    if (llr_dtype != LDPC5G_F32 && !(llr_dtype == LDPC5G_F64 && mod == 1 && sym_dtype == LDPC5G_F64))
        return fail(LDPC5G_ESIZE, "float64 LLRs only for BPSK on complex128 symbols (demod_bpsk.py)");
    if (T < 0 || nsym < 0) return fail(LDPC5G_ESIZE, "bad sizes");
    if (T > 1 && (ldsym < nsym || ldnv < nsym || ldllr < nsym * Qm || (prbs && ldw < (nsym * Qm + 31) / 32)))
        return fail(LDPC5G_ESIZE, "bad strides");
    if (T == 0 || nsym == 0) return LDPC5G_OK;
    if (!sym || !noise_var || !llr) return fail(LDPC5G_ESIZE, "null buffer");
    const dim3 grid((unsigned)((nsym + 255) / 256), T), blk(256);
    hipStream_t st = (hipStream_t)stream;
    const double A = 1.0 / sqrt((double)mod_scale(Qm));   // A = 1/math.sqrt(scale) (demod_*.py)
#define LDPC5G_DEMOD(QM, PI2, TIN, TOUT)                                                          \
    hipLaunchKernelGGL((demod_descramble_kernel<QM, PI2, TIN, TOUT>), grid, blk, 0, st,         \
                       (const TIN*)sym, ldsym, noise_var, ldnv, prbs, ldw, nsym, A, (TOUT*)llr, ldllr)
#define LDPC5G_DEMOD_ALL(TIN)                               \
    switch (mod) {                                          \
        case -1: LDPC5G_DEMOD(1, true, TIN, float); break;  \
        case 1: LDPC5G_DEMOD(1, false, TIN, float); break;  \
        case 2: LDPC5G_DEMOD(2, false, TIN, float); break;  \
        case 4: LDPC5G_DEMOD(4, false, TIN, float); break;  \
        case 6: LDPC5G_DEMOD(6, false, TIN, float); break;  \
        case 8: LDPC5G_DEMOD(8, false, TIN, float); break;  \
        default: LDPC5G_DEMOD(10, false, TIN, float); break; \
    }
    if (llr_dtype == LDPC5G_F64) LDPC5G_DEMOD(1, false, double2, double);
    else if (sym_dtype == LDPC5G_F32) { LDPC5G_DEMOD_ALL(float2) }
    else { LDPC5G_DEMOD_ALL(double2) }
#undef LDPC5G_DEMOD_ALL
#undef LDPC5G_DEMOD
    return check_hip(hipGetLastError(), "demod_descramble launch");
}

}  // extern "C"
