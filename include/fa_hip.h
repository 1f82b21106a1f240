/*
 * fa_hip.h — C ABI of libfa_hip.so, the MI355X (gfx950) FlashAttention library.
 *
 * This is the drop-in boundary for the reference's pybind11 module `flash_attn_cuda`
 * (reference: setup.py:117-121). Each entry point replaces one reference interface:
 *
 *   fa_fwd  <- flash_attn_cuda.fwd  = mha_fwd   (csrc/flash_attn/fmha_api.cpp:112-242,
 *                                                  bound at fmha_api.cpp:244-247)
 *   fa_bwd  <- flash_attn_cuda.bwd              (called at flash_attn/flash_attn_interface.py:31-33;
 *                                                  never bound in the reference, built fresh here)
 *   fa_fwd_block <- flash_attn_cuda.fwd_block (called at flash_attn/flash_blocksparse_attn_interface.py:46-48;
 *   fa_bwd_block <- flash_attn_cuda.bwd_block  flash_attn/flash_blocksparse_attn_interface.py:55-58;
 *                                               declared by the reference's Python but never bound
 *                                               natively, built fresh here)
 *   fa_index_first_axis     <- IndexFirstAxis.forward / IndexPutFirstAxis.backward
 *                              (flash_attn/bert_padding.py:11-38, 56-61)
 *   fa_index_put_first_axis <- IndexPutFirstAxis.forward / IndexFirstAxis.backward
 *                              (flash_attn/bert_padding.py:41-55, 25-38); with unpad_input /
 *                              pad_input (:99-134) on top
 *   fa_index_add_first_axis <- IndexFirstAxisResidual.backward (flash_attn/bert_padding.py:82-94)
 *   fa_rotary               <- apply_rotary_pos_emb + RotaryEmbedding(2D).forward and their autograd
 *                              backward (flash_attn/rotary.py:22-41, 86-135)
 *   (fa_fwd runs hand-scheduled gfx950 assembly kernels, csrc/asm/gen_fwd.py, embedded in the library
 *    as code objects, for head_dim ≤ 64 (≤ 32: the D = 32 tile), 80, 96 or 128, fp16/bf16, causal or not, no dropout, dense,
 *    no fused rotary; the persistent form for non-causal grids with more blocks than CUs; every form
 *    computes fp32-exact scores; fa_asm.cpp fwd_asm_eligible / persistent_grid_for).
 *    FaFwdArgs.impl selects a form or the HIP kernels.)
 *   fa_query, fa_last_error, fa_version, fa_fwd_kernel_name: host helpers (no reference counterpart; the reference
 *                                                  raised through TORCH_CHECK / exit(1),
 *                                                  fmha_api.cpp:131-170, fmha_utils.h:36-48)
 *
 * Conventions:
 *   - Plain C types only: raw device pointers, element strides (int64), sizes. No torch types.
 *   - The caller allocates every output and workspace (the Python layer uses torch.empty).
 *   - Every call is stream-ordered and asynchronous on `stream` (a hipStream_t, NULL = default).
 *     No host synchronisation, no device allocation, no exit(), so calls can be captured into a
 *     hipGraph. One-time state: the first assembly-kernel call on a device loads all of that
 *     device's code objects (hipModuleLoadData, under a mutex, capture mode exchanged to relaxed);
 *     if that first call is inside a capture and the load fails, FA_IMPL_AUTO runs the HIP kernels
 *     instead. One eager call before capturing avoids both. Dropout under capture: a captured (seed, rng_offset) is a constant, so pass
 *     rng_offset_dev pointing at a device word that the graph advances before each launch
 *     (flash_attn_hip.py does this), or every replay draws the same mask.
 *   - Return 0 on success; non-zero = error, with a message in fa_last_error() (thread-local).
 *   - The only global mutable state is that per-device code-object table (mutex-guarded) and the
 *     cached CU count: concurrent calls from several host threads are safe.
 *
 * Layout ("unpadded", reference fmha_api.cpp:113-115,149-151): q is (total_q, H, D), k/v are
 * (total_k, H, D), with stride(-1) == 1 and arbitrary row/head strides (packed qkv/kv views).
 * Sequences are delimited by int32 cu_seqlens (B+1) on the device.
 */
#ifndef FA_HIP_H_
#define FA_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { FA_DTYPE_FP16 = 0, FA_DTYPE_BF16 = 1, FA_DTYPE_FP32 = 2 /* padding helpers only */ };

/* Error codes. */
enum {
    FA_OK = 0,
    FA_ERR_INVALID_ARGUMENT = 1,
    FA_ERR_UNSUPPORTED = 2,
    FA_ERR_LAUNCH = 3,
};

/* Forward arguments. Mirrors mha_fwd's parameters (fmha_api.cpp:112-125) plus the
 * pointers/strides that set_params_fprop fills (fmha_api.cpp:38-110). */
typedef struct FaFwdArgs {
    const void *q;            /* (total_q, H, D) fp16/bf16 */
    const void *k;            /* (total_k, H, D) */
    const void *v;            /* (total_k, H, D) */
    void *o;                  /* (total_q, H, D) output, same dtype */
    float *softmax_lse;       /* (B, H, lse_stride) fp32 output; natural-log LSE of scaled scores */
    void *s_dmask;            /* optional (B, H, s_rows, s_cols) probabilities, dtype of q; NULL = off */
    const int32_t *cu_seqlens_q;  /* (B+1) device */
    const int32_t *cu_seqlens_k;  /* (B+1) device */
    int64_t q_row_stride, q_head_stride;   /* element strides */
    int64_t k_row_stride, k_head_stride;
    int64_t v_row_stride, v_head_stride;
    int64_t o_row_stride, o_head_stride;
    int32_t batch;            /* B */
    int32_t nheads;           /* H */
    int32_t head_dim;         /* D: multiple of 8, <= 128 (fmha_api.cpp:158) */
    int32_t max_seqlen_q;
    int32_t max_seqlen_k;
    int32_t lse_stride;       /* >= max_seqlen_q (the Python layer uses round16(max_seqlen_q)) */
    int32_t s_rows, s_cols;   /* s_dmask extents (>= max_seqlen_q, >= max_seqlen_k) */
    float softmax_scale;
    float p_dropout;          /* probability of DROPPING, in [0, 1) (fmha_api.cpp:99-107) */
    uint64_t rng_seed;        /* Philox key */
    uint64_t rng_offset;      /* Philox stream offset reserved from the torch generator */
    const uint64_t *rng_offset_dev;  /* optional device word added to rng_offset when the kernel
                                        runs (NULL = none): lets a captured hipGraph advance the
                                        dropout stream on every replay */
    int32_t is_causal;        /* top-left aligned: col <= row (mask.h:58-72) */
    int32_t dtype;            /* FA_DTYPE_* */
    /* Optional rotary embedding fused into the Q load (flash_attn/rotary.py:31-41, README.md:56
     * "Fuse rotary embedding"): when rot_cos != NULL, row r of each query sequence is rotated
     * with table row r before QK^T, rounded exactly as fa_rotary's separate pass (so the result
     * equals fa_rotary followed by fa_fwd bit for bit). k must already be rotated. Tables are
     * (>= max_seqlen_q, rot_stride) in q's dtype, rot_stride >= head_dim. NULL = off. */
    const void *rot_cos;
    const void *rot_sin;
    int64_t rot_stride;
    /* Kernel family (FA_IMPL_*). FA_IMPL_AUTO picks the fastest kernel for the shape: the
     * hand-scheduled assembly forward for head_dim ≤ 64 (≤ 32: the D = 32 tile), 80, 96 or 128, fp16/bf16, no dropout,
     * dense, no fused rotary (non-causal grids with more blocks than CUs take its persistent form); the
     * HIP kernels otherwise. FA_IMPL_HIP forces the HIP kernels; FA_IMPL_ASM4 / FA_IMPL_ASM4P force
     * the one-wave-per-SIMD assembly form, one workgroup per block or persistent, where the shape is
     * eligible. The assembly forms compute the same fp32-exact scores and sums in the same order
     * (bitwise equal outputs); the HIP kernels differ from them in the last bits (summation order),
     * all within the reference's 2x rule. FA_IMPL_ASM8 (the two-waves-per-SIMD form, an A/B build of
     * the generator since round 6) is reserved: fa_fwd rejects it with FA_ERR_INVALID_ARGUMENT. */
    int32_t impl;
    int32_t reserved;         /* 0 */
} FaFwdArgs;

enum { FA_IMPL_AUTO = 0, FA_IMPL_HIP = 1, FA_IMPL_ASM4 = 2, FA_IMPL_ASM8 = 3, FA_IMPL_ASM4P = 4 };

/* Backward arguments. Mirrors the bwd call made by flash_attn_interface.py:31-33:
 * bwd(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_q, cu_k, max_q, max_k, p, scale,
 *     zero_tensors, causal, gen) -> softmax_d. */
typedef struct FaBwdArgs {
    const void *dout;         /* (total_q, H, D) */
    const void *q;
    const void *k;
    const void *v;
    const void *out;          /* forward output */
    const float *softmax_lse; /* (B, H, lse_stride) from fa_fwd */
    void *dq;                 /* (total_q, H, D) output; may be a strided view (qkv-packed) */
    void *dk;                 /* (total_k, H, D) output; may be a strided view */
    void *dv;
    float *softmax_d;         /* (B, H, lse_stride) fp32 output: rowsum(dout * out) */
    float *dq_accum;          /* workspace: fa_query(FA_QUERY_BWD_WORKSPACE) bytes, any contents;
                                 may be NULL when fa_query(FA_QUERY_BWD_WORKSPACE_NEEDED) is 0 */
    const int32_t *cu_seqlens_q;
    const int32_t *cu_seqlens_k;
    int64_t do_row_stride, do_head_stride;
    int64_t q_row_stride, q_head_stride;
    int64_t k_row_stride, k_head_stride;
    int64_t v_row_stride, v_head_stride;
    int64_t o_row_stride, o_head_stride;
    int64_t dq_row_stride, dq_head_stride;
    int64_t dk_row_stride, dk_head_stride;
    int64_t dv_row_stride, dv_head_stride;
    int32_t batch, nheads, head_dim, max_seqlen_q, max_seqlen_k;
    int32_t total_q;          /* rows of q / dq */
    int32_t lse_stride;
    float softmax_scale;
    float p_dropout;
    uint64_t rng_seed;        /* must equal the forward's seed/offset to replay its dropout mask */
    uint64_t rng_offset;
    const uint64_t *rng_offset_dev;  /* as in FaFwdArgs: must be the forward's word, unchanged since */
    int32_t is_causal;
    int32_t dtype;
} FaBwdArgs;

/* Block-sparsity layout for fa_fwd_block / fa_bwd_block: the 0/1 "blockmask" of the
 * reference (flash_attn/flash_blocksparse_attn_interface.py:8-40 before convert_blockmask;
 * semantics of tests/test_flash_attn.py:189-215): mask[r][c] != 0 lets query rows
 * 16r..16r+15 attend keys 256c..256c+255 (positions within each sequence). Rows with no live
 * block produce output 0 and lse -inf. */
typedef struct FaBlockMask {
    const uint8_t *mask;      /* (rows, cols) bytes on the device */
    int64_t row_stride;       /* elements between consecutive rows (>= cols) */
    int32_t rows;             /* >= ceil(max_seqlen_q / 16) */
    int32_t cols;             /* >= ceil(max_seqlen_k / 256), <= 64 */
} FaBlockMask;

/* Forward pass. Writes o, softmax_lse and (if s_dmask != NULL) the attention probabilities
 * softmax(QK^T*scale) in row-major (B, H, s_rows, s_cols), with dropped entries negated
 * (the sign convention of the reference, softmax.h:256-296). */
int fa_fwd(const FaFwdArgs *args, void *stream);

/* Backward pass. Writes dq, dk, dv and softmax_d. */
int fa_bwd(const FaBwdArgs *args, void *stream);

/* Block-sparse forward / backward: as fa_fwd / fa_bwd with the layout `mask` applied on top of
 * the key-length and causal masks. Blocks that are 0 for every row of a workgroup are skipped
 * (no loads, no MFMAs). Limits: mask->cols <= 64 (max_seqlen_k <= 16384),
 * max_seqlen_q <= 32768. */
int fa_fwd_block(const FaFwdArgs *args, const FaBlockMask *mask, void *stream);
int fa_bwd_block(const FaBwdArgs *args, const FaBlockMask *mask, void *stream);

/* Var-len packing (bert_padding). Rows of `row_bytes` bytes, byte strides, int64 row indices on
 * the device. Indices outside the valid range read as zero rows / are ignored.
 *   fa_index_first_axis:     dst[i] = src[indices[i]]                  for i < n
 *   fa_index_put_first_axis: dst = 0; dst[indices[i]] = src[i]         (every dst row written once;
 *                            workspace: fa_query(FA_QUERY_PAD_WORKSPACE, dst_rows) bytes)
 *   fa_index_add_first_axis: dst[indices[i]] += src[i] elementwise in `dtype` (FA_DTYPE_*, fp32
 *                            allowed); indices must be unique. */
int fa_index_first_axis(const void *src, int64_t src_rows, int64_t src_row_stride, const int64_t *indices, int64_t n,
                        void *dst, int64_t dst_row_stride, int64_t row_bytes, void *stream);
int fa_index_put_first_axis(const void *src, int64_t src_row_stride, const int64_t *indices, int64_t n, void *dst,
                            int64_t dst_rows, int64_t dst_row_stride, int64_t row_bytes, int32_t *workspace,
                            void *stream);
int fa_index_add_first_axis(const void *src, int64_t src_row_stride, const int64_t *indices, int64_t n, void *dst,
                            int64_t dst_rows, int64_t dst_row_stride, int64_t row_elems, int32_t dtype,
                            void *stream);

/* Rotary position embedding (flash_attn/rotary.py:22-41): y = x*cos + rotate_half(x)*sin with
 * interleaved pairs (2i, 2i+1), every product and the sum rounded to the 16-bit dtype as torch's
 * eager evaluation does (bit-identical to the reference). inverse = 1 applies the autograd
 * transpose (the backward). x, y: (B, S, NSLOT, H, D), element strides, stride(-1) == 1, 16-byte
 * aligned rows; y may alias x. Slots [0, nrot) are rotated; the others are copied when y != x.
 * cos/sin: (>= S, D) tables in x's dtype (position = index along S). */
typedef struct FaRotaryArgs {
    const void *x;
    void *y;
    const void *cos;
    const void *sin;
    int64_t x_strides[4];     /* batch, seq, slot, head (elements) */
    int64_t y_strides[4];
    int64_t table_stride;     /* elements between table rows */
    int32_t batch, seqlen, nslot, nheads, head_dim;
    int32_t nrot;
    int32_t inverse;
    int32_t dtype;            /* FA_DTYPE_FP16 / FA_DTYPE_BF16 */
} FaRotaryArgs;
int fa_rotary(const FaRotaryArgs *args, void *stream);

enum {
    FA_QUERY_BWD_WORKSPACE = 1,   /* a = total_q, b = nheads, c = head_dim -> bytes */
    FA_QUERY_MAX_HEAD_DIM = 2,    /* -> 128 */
    FA_QUERY_RNG_INCREMENT = 3,   /* Philox offset increment a forward reserves per call */
    FA_QUERY_FWD_ARGS_SIZE = 4,   /* sizeof(FaFwdArgs): lets FFI bindings check their struct layout */
    FA_QUERY_BWD_ARGS_SIZE = 5,   /* sizeof(FaBwdArgs) */
    FA_QUERY_MASK_ARGS_SIZE = 6,  /* sizeof(FaBlockMask) */
    FA_QUERY_PAD_WORKSPACE = 7,   /* a = dst_rows -> bytes of fa_index_put_first_axis's workspace */
    FA_QUERY_ROTARY_ARGS_SIZE = 8,   /* sizeof(FaRotaryArgs) */
    FA_QUERY_BWD_WORKSPACE_NEEDED = 9,   /* a = head_dim, b = (p_dropout > 0), c = block-sparse
                                            -> 1 if fa_bwd reads dq_accum, 0 if dq is written directly */
    FA_QUERY_ASM_LAUNCHES = 10,   /* -> assembly-forward launches this process has enqueued or captured
                                     (diagnostics: which kernel family a call, or a graph capture, took) */
};
int64_t fa_query(int what, int64_t a, int64_t b, int64_t c);

/* Last error message of the calling host thread ("" if none). */
const char *fa_last_error(void);

/* Library version string. */
const char *fa_version(void);

/* Name of the GPU kernel fa_fwd would launch for these arguments: an assembly kernel's symbol exactly
 * as a rocprofv3 kernel trace shows it (e.g. "fa_fwd_d64p_bf16_asm"), or for the HIP template family
 * the prefix of its demangled name in that trace ("fa::fa_fwd_kernel<64," of
 * "void fa::fa_fwd_kernel<64, fa::Bf16, ...>(...)"). NULL when fa_fwd would reject the arguments or
 * launch nothing (max_seqlen_q == 0). Launches nothing (host helper, like fa_query; used by bench.py
 * to name the kernel its roofline measures). */
const char *fa_fwd_kernel_name(const FaFwdArgs *args);

#ifdef __cplusplus
}
#endif

#endif /* FA_HIP_H_ */
