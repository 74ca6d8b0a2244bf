/*
 * ldpc5g.h — C ABI of the MI355X-native 5G NR LDPC engine (libldpc5g.so, gfx950).
 *
 * The engine replaces the hot path of the reference py5gphy/ldpc package:
 *   ldpc5g_encode        <- py5gphy/ldpc/nr_ldpc_encode.py:8     encode_ldpc(ck, bgn)
 *                           (+ _gen_ldpc_parity_bit :52-115), batched over codeblocks
 *   ldpc5g_decode_ms     <- py5gphy/ldpc/nr_ldpc_decode.py:11    nr_decode_ldpc(LLRin, Zc, bgn, L,
 *                           'min-sum', alpha, beta) and decode_ldpc :51-143 / _min_sum_process
 *                           :178-227, batched over codeblocks
 *   ldpc5g_decode_ms_mixed  the same over a batch of codeblocks with per-codeblock (bgn, Zc),
 *                           the shape DLSCHDecode (py5gphy/nr_pdsch/nr_dlsch_decode.py:62-91)
 *                           and ULSCH_decoding (py5gphy/nr_pusch/nr_ulsch_decode.py:92) feed
 *   ldpc5g_find_ils      <- py5gphy/ldpc/ldpc_info.py:81         find_iLS(Zc)
 *
 * Conventions
 *   - All buffer pointers are DEVICE pointers (hipMalloc / torch tensors); the library never
 *     allocates or frees caller buffers.  `stream` is a hipStream_t (NULL = default stream).
 *   - Bits are int8 per bit (0/1, -1 = filler), LLRs are log(P0/P1) (positive => bit 0).
 *   - Calls are asynchronous on `stream` and reentrant; ldpc5g_last_error() is thread-local.
 *   - Return 0 on success, or a negative code: the Python host maps them to AssertionError,
 *     as the reference's `assert` checks (nr_ldpc_encode.py:18,29; nr_ldpc_decode.py:23-37).
 */
#ifndef LDPC5G_H
#define LDPC5G_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC5G_OK 0
#define LDPC5G_EBGN (-1)   /* bgn not in {1,2}                                 */
#define LDPC5G_EZC (-2)    /* Zc not a TS 38.212 lifting size (find_iLS == 255) */
#define LDPC5G_ESIZE (-3)  /* bad batch / stride / L / dtype / schedule        */
#define LDPC5G_EHIP (-4)   /* HIP runtime error (launch failure)               */

/* LLR element types */
#define LDPC5G_F64 0       /* float64: bit-exact with the reference's numpy float64 decoder */
#define LDPC5G_F32 1       /* float32 */

/* decode flags */
#define LDPC5G_LLR_FULL 1  /* LLR rows hold all Nf = 68Zc/52Zc columns, the 2Zc punctured ones
                              included (decode_ldpc(LLRin, H, ...) input, nr_ldpc_decode.py:51) */

/* decoding schedules */
#define LDPC5G_FLOODING 0  /* the reference's two-phase (Jacobi) schedule, nr_ldpc_decode.py:105-131 */
#define LDPC5G_LAYERED 1   /* row-block serial schedule (perf mode, float32 only)                  */

/* Lifting-set index 0..7 of Zc (TS 38.212 Table 5.3.2-1), 255 if Zc is not a lifting size. */
int ldpc5g_find_ils(int32_t Zc);

/* Encode B codeblocks.
 *   ck : [B][ldk] int8, first K = 22*Zc (bgn 1) / 10*Zc (bgn 2) entries used, values 0/1/-1
 *   dn : [B][ldn] int8, first N = 66*Zc / 50*Zc entries written:
 *        dn[0:K-2Zc] = ck[2Zc:K] (fillers stay -1), dn[K-2Zc:N] = parity bits.
 *   Parity treats ck[k] = -1 (k >= 2Zc) as 0, exactly as the reference zeroes fillers before
 *   encoding.  ck is not modified (the reference's in-place filler zeroing is done host-side). */
int ldpc5g_encode(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc,
                  int64_t ldk, int64_t ldn, void* stream);

/* Min-sum decode (MS / normalized alpha<1 / offset beta>0 / mixed) of B codeblocks.
 *   llr    : [B][ldl] of llr_dtype, N = 66*Zc / 50*Zc entries (2*Zc systematic bits punctured,
 *            decoded with LLR 0), or Nf = 68*Zc / 52*Zc entries when flags & LDPC5G_LLR_FULL
 *   ck     : [B][ldc] int8, Nf = 68*Zc / 52*Zc hard decisions written (blkandcrc = ck[0:K])
 *   status : [B] uint8, 1 iff ck satisfies every parity check
 *   iters  : [B] int32, check-node updates performed (flooding: the reference's loop index at
 *            its early return, else L; layered: iterations run)
 *   schedule LDPC5G_FLOODING works with F64 (bit-exact with the reference) and F32;
 *   LDPC5G_LAYERED requires F32. */
int ldpc5g_decode_ms(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L,
                     double alpha, double beta, int32_t schedule, int32_t flags, int64_t ldl,
                     int64_t ldc, void* stream);

/* Hard-decision bit flipping (algo='BF')  <- py5gphy/ldpc/ldpc_decoder_bit_flipping.py:5-73
 * reached through nr_decode_ldpc(..., algo='BF') (nr_ldpc_decode.py:65-67).  Same buffers as
 * ldpc5g_decode_ms; ck holds the 0/1 decisions (the reference returns them as float64), status
 * is 0 after L iterations without a zero syndrome (the reference checks only at loop start). */
int ldpc5g_decode_bf(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L,
                     int32_t flags, int64_t ldl, int64_t ldc, void* stream);

/* Float64 sum-product, flooding (algo='BP')  <- nr_ldpc_decode.py:51-143 + _BP_process :145-176.
 * Per-edge messages do not compress: the caller provides a float64 device scratch of
 * ldpc5g_bp_scratch_elems(B, bgn, Zc) elements (-1 on bad arguments). */
int64_t ldpc5g_bp_scratch_elems(int32_t B, int32_t bgn, int32_t Zc);
int ldpc5g_decode_bp(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                     double* scratch, int64_t scratch_elems, int32_t B, int32_t bgn, int32_t Zc,
                     int32_t L, int32_t flags, int64_t ldl, int64_t ldc, void* stream);

/* One codeblock of a mixed batch: base graph, lifting size, element offsets of its LLR row
 * (into llr_base, in elements) and of its ck row (into ck_base, in bytes). */
typedef struct {
    int32_t bgn;
    int32_t Zc;
    int64_t llr_off;
    int64_t ck_off;
} ldpc5g_cb_desc_t;

/* Decode a batch of codeblocks with heterogeneous (bgn, Zc) in at most two launches (one per
 * base graph).  `desc` is a HOST array of B descriptors; status[b] / iters[b] follow desc order.
 * The library keeps a small internal device work list (grown on demand, one per device). */
int ldpc5g_decode_ms_mixed(const ldpc5g_cb_desc_t* desc, int32_t B, const void* llr_base,
                           int32_t llr_dtype, int8_t* ck_base, uint8_t* status, int32_t* iters,
                           int32_t L, double alpha, double beta, int32_t schedule,
                           int32_t flags, void* stream);

/* Message of the last failed call on this thread ("" if none). */
const char* ldpc5g_last_error(void);

/* Library version string. */
const char* ldpc5g_version(void);

/* Diagnostics: decoder workgroups that can be resident on one CU (HIP occupancy calculator) for
 * (bgn, llr_dtype, schedule).  No reference counterpart. */
int ldpc5g_dec_blocks_per_cu(int32_t bgn, int32_t llr_dtype, int32_t schedule);

#ifdef __cplusplus
}
#endif

#endif /* LDPC5G_H */
