/* A plain C caller of the C ABI (include/fa_hip.h), the way a non-Python binding would use it:
 * device buffers from the HIP runtime, FaFwdArgs/FaBwdArgs filled by hand, fa_fwd + fa_bwd on the
 * default stream, results copied back. It prints the outputs' checksums and the first values so
 * tests/test_c_caller.py can compare them with the Python path on the same inputs.
 *
 *   gcc -std=c11 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include tests/c_caller/fa_c_caller.c \
 *       -L <libdir> -lfa_hip -L /opt/rocm/lib -lamdhip64 -lm -o fa_c_caller
 *   ./fa_c_caller <B> <H> <S> <D> <causal> <inputs.bin> <outputs.bin>
 * inputs.bin: q, k, v, dout as bf16 (B*S, H, D) each; outputs.bin: o, dq, dk, dv (bf16) + lse (fp32).
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fa_hip.h"

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 2;                                                             \
        }                                                                         \
    } while (0)

int main(int argc, char **argv) {
    if (argc != 8) {
        fprintf(stderr, "usage: %s B H S D causal inputs.bin outputs.bin\n", argv[0]);
        return 1;
    }
    const int B = atoi(argv[1]), H = atoi(argv[2]), S = atoi(argv[3]), D = atoi(argv[4]), causal = atoi(argv[5]);
    const size_t n = (size_t)B * S * H * D, bytes = n * 2, lse_stride = (S + 15) / 16 * 16;
    unsigned short *host = (unsigned short *)malloc(4 * bytes);
    FILE *f = fopen(argv[6], "rb");
    if (!f || fread(host, 1, 4 * bytes, f) != 4 * bytes) { fprintf(stderr, "bad inputs\n"); return 1; }
    fclose(f);
    void *q, *k, *v, *dout, *o, *dq, *dk, *dv, *lse, *softmax_d, *ws;
    int *cu;
    CHECK(hipMalloc(&q, bytes)); CHECK(hipMalloc(&k, bytes)); CHECK(hipMalloc(&v, bytes)); CHECK(hipMalloc(&dout, bytes));
    CHECK(hipMalloc(&o, bytes)); CHECK(hipMalloc(&dq, bytes)); CHECK(hipMalloc(&dk, bytes)); CHECK(hipMalloc(&dv, bytes));
    CHECK(hipMalloc(&lse, (size_t)B * H * lse_stride * 4)); CHECK(hipMalloc(&softmax_d, (size_t)B * H * lse_stride * 4));
    CHECK(hipMalloc(&ws, (size_t)fa_query(FA_QUERY_BWD_WORKSPACE, (int64_t)B * S, H, D)));
    CHECK(hipMalloc((void **)&cu, (B + 1) * sizeof(int)));
    int *cu_h = (int *)malloc((B + 1) * sizeof(int));
    for (int b = 0; b <= B; ++b) cu_h[b] = b * S;
    CHECK(hipMemcpy(cu, cu_h, (B + 1) * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(q, host, bytes, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(k, host + n, bytes, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(v, host + 2 * n, bytes, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dout, host + 3 * n, bytes, hipMemcpyHostToDevice));

    FaFwdArgs a;
    memset(&a, 0, sizeof(a));
    a.q = q; a.k = k; a.v = v; a.o = o; a.softmax_lse = (float *)lse;
    a.cu_seqlens_q = cu; a.cu_seqlens_k = cu;
    a.q_row_stride = a.k_row_stride = a.v_row_stride = a.o_row_stride = (int64_t)H * D;
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = D;
    a.batch = B; a.nheads = H; a.head_dim = D; a.max_seqlen_q = S; a.max_seqlen_k = S;
    a.lse_stride = (int32_t)lse_stride; a.softmax_scale = 1.0f / sqrtf((float)D);
    a.is_causal = causal; a.dtype = FA_DTYPE_BF16;
    if (fa_fwd(&a, NULL) != 0) { fprintf(stderr, "fa_fwd: %s\n", fa_last_error()); return 3; }

    FaBwdArgs g;
    memset(&g, 0, sizeof(g));
    g.dout = dout; g.q = q; g.k = k; g.v = v; g.out = o; g.softmax_lse = (float *)lse;
    g.dq = dq; g.dk = dk; g.dv = dv; g.softmax_d = (float *)softmax_d; g.dq_accum = (float *)ws;
    g.cu_seqlens_q = cu; g.cu_seqlens_k = cu;
    g.do_row_stride = g.q_row_stride = g.k_row_stride = g.v_row_stride = g.o_row_stride = (int64_t)H * D;
    g.dq_row_stride = g.dk_row_stride = g.dv_row_stride = (int64_t)H * D;
    g.do_head_stride = g.q_head_stride = g.k_head_stride = g.v_head_stride = g.o_head_stride = D;
    g.dq_head_stride = g.dk_head_stride = g.dv_head_stride = D;
    g.batch = B; g.nheads = H; g.head_dim = D; g.max_seqlen_q = S; g.max_seqlen_k = S;
    g.total_q = B * S; g.lse_stride = (int32_t)lse_stride; g.softmax_scale = a.softmax_scale;
    g.is_causal = causal; g.dtype = FA_DTYPE_BF16;
    if (fa_bwd(&g, NULL) != 0) { fprintf(stderr, "fa_bwd: %s\n", fa_last_error()); return 3; }
    CHECK(hipDeviceSynchronize());

    unsigned short *out = (unsigned short *)malloc(4 * bytes);
    float *lse_h = (float *)malloc((size_t)B * H * lse_stride * 4);
    CHECK(hipMemcpy(out, o, bytes, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(out + n, dq, bytes, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(out + 2 * n, dk, bytes, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(out + 3 * n, dv, bytes, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(lse_h, lse, (size_t)B * H * lse_stride * 4, hipMemcpyDeviceToHost));
    f = fopen(argv[7], "wb");
    fwrite(out, 1, 4 * bytes, f);
    fwrite(lse_h, 4, (size_t)B * H * lse_stride, f);
    fclose(f);
    printf("ok %s\n", fa_version());
    return 0;
}
