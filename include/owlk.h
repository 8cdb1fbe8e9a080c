/* libowlk -- MI355X (gfx950) kernels for the owl_wms DiT/MMDiT training hot path.
 *
 * C ABI: plain device pointers, int64 sizes/strides (elements), a hipStream_t passed as void*.
 * Every entry point only enqueues work on `stream`; none allocates, frees or synchronises.
 * Return value: 0 = ok; 1 = argument error; 2 = HIP launch error.  owlk_last_error() returns a
 * thread-local message for the last failure.  bf16 buffers are 16-byte aligned with row strides
 * that are multiples of 8 elements.
 *
 * Each entry cites the reference interface it replaces (paths relative to the reference repo).
 */
#ifndef OWLK_H
#define OWLK_H
#ifdef __cplusplus
extern "C" {
#endif

const char* owlk_last_error(void);
int owlk_version(void);
int owlk_device_ok(void);

/* ---- GEMM (replaces every nn.Linear / cuBLAS call on the hot path: attn.py:72-73,82,113;
 *      mlp.py:29-37; modulation.py:11,32; gamerft.py:26-27; and the X@X.mT / A@A / B@X products
 *      of muon.py:31-34).
 *   C[m, n] = epi( sum_k A(m, k) * B(n, k) ),  A(m,k) = a_trans ? A[k*lda+m] : A[m*lda+k],
 *                                               B(n,k) = b_trans ? B[k*ldb+n] : B[n*ldb+k]
 *   epi 0 STORE      C = alpha*acc + bf16(bias[n]) + beta*C           (bf16 or fp32 C)
 *       1 SILU       aux = bf16(acc + bias); C = bf16(silu(aux))
 *       2 GATE_RESID aux = y = bf16(acc + bias); C = bf16(resid + bf16(gate[m / tpf, n] * y))
 *       3 DSILU      C = bf16(bf16(acc) * silu'(aux)); a non-null resid is an OUTPUT here:
 *                    resid = bf16(silu(aux)) (the activation a lean backward did not keep)
 *       4 AXPBY      C = bf16(bf16(alpha * bf16(acc)) + bf16(beta * aux))
 *       5 SCALE2     C = bf16(acc); aux = bf16(alpha * bf16(acc))   (a_trans = b_trans = 0 only)
 *   batch: blockIdx.z with element strides sA, sB, sC, sAux, sGate, sRes.
 *   fp32 STORE with beta 0 or 1 and K >= 8192 onto a small output (weight gradients) splits K
 *   over workgroups.  With a caller-owned workspace of owlk_gemm_ws_bytes(...) bytes (ws, 16-B
 *   aligned) the per-split partials go there and one fixed-order reduce forms C: the result is
 *   bitwise deterministic.  Without it (ws null or too small) the splits combine by fp32 atomics
 *   onto C (cleared first when beta = 0).  The library never allocates.
 *   Decode plan (M <= 128, batch 1, a_trans = b_trans = 0, bf16 C, STORE / SILU / GATE_RESID,
 *   N % 64 == 0, K % 32 == 0): one launch of 64-column tiles with K split over workgroups; the last
 *   workgroup of a tile adds the chunks' partials in order (deterministic).  When
 *   owlk_gemm_ws_bytes reports a non-zero size for it, the first OWLK_DECODE_COUNTER_BYTES of ws
 *   are per-tile arrival counters that MUST be zero on entry; every launch leaves them zero, so
 *   keep one zero-initialised workspace per device and do not share it between concurrent
 *   streams.  Without a large enough workspace the call takes the 64^2-tile path.
 *   colsum (optional, batch 1, bf16 C): colsum[n] += sum_m C[m, n] over the stored bf16 values
 *   (bias gradient of the next layer, fused into the DSILU epilogue of the 256^2 kernel; a
 *   separate column-sum pass otherwise); deterministic with the workspace (per-tile partial rows
 *   added in order), fp32 atomics without.  It accumulates onto colsum. */
#define OWLK_DECODE_COUNTER_BYTES 4096
int owlk_gemm(long M, long N, long K, long batch,
              const void* A, long lda, long sA, int a_trans,
              const void* B, long ldb, long sB, int b_trans,
              void* C, long ldc, long sC, int c_f32,
              int epi, float alpha, float beta, const float* bias,
              void* aux, long ldaux, long sAux,
              const void* gate, long ldgate, long sGate, long tpf,
              const void* resid, long ldres, long sRes,
              float* colsum, void* ws, long ws_bytes, void* stream);
/* owlk_gemm (batch 1, no colsum) with frame-strided operand rows: with x_fs > 0, row r of that operand
 *   lives at (r / OWLK_FRAME_ROWS) * x_fs + (r % OWLK_FRAME_ROWS) * ldx elements (the rows of A / B are
 *   its m / n rows, or its k rows when transposed; C's are m).  The video rows of the MMDiT joint
 *   sequence -- frame f = [64 video | 1 audio] tokens, mmattn.py:54-60 -- are read and written in
 *   place (x_fs = 65 * ldx) with no interleave / split copies.  256^2-tile shapes only (M, N multiples
 *   of 256 where tiled, K % 64 == 0; split-K weight gradients need the workspace); C frame-strided only
 *   for a bf16 STORE; otherwise returns 1. */
#define OWLK_FRAME_ROWS 64
int owlk_gemm_frames(long M, long N, long K, const void* A, long lda, long a_fs, int a_trans,
                     const void* B, long ldb, long b_fs, int b_trans, void* C, long ldc, long c_fs,
                     int c_f32, int epi, float alpha, float beta, const float* bias, void* aux, long ldaux,
                     const void* gate, long ldgate, long tpf, const void* resid, long ldres, void* ws,
                     long ws_bytes, void* stream);
/* dO = dY W^T-layout product of the attention output projection's backward (attn.py:113: dY [M, K] bf16,
 *   W [K, N] bf16 rows = the out-projection weight [out, in], bf16 dO [M, N]) AND the flash-attention
 *   backward's delta[b, h, t] = sum_c dO[b L + t, h D + c] * O[b L + t, h D + c] (fp32 [M / L, H, L], as
 *   owlk_attn_delta) in one launch when the shape takes the 256^2 ping-pong kernel at D = 64 (the
 *   delta from the stored bf16 dO in owlk_attn_delta's order: the same bits); otherwise owlk_gemm +
 *   owlk_attn_delta (then ldo must equal ldc).  N = H * D, M % L == 0. */
int owlk_gemm_attn_delta(long M, long N, long K, const void* dY, long lddy, const void* W, long ldw, void* dO,
                         long ldc, const void* o, long ldo, long L, int H, int D, float* delta, void* stream);
/* qkv = A W^T + bias (the qkv projection, attn.py:82: A [M, K] bf16, W [N, K] bf16, N = 3 H D, bf16 qkv)
 *   AND owlk_qk_rope_fwd of its q | k columns into out / rstd (same tables, positions and checks) in one
 *   launch when the shape takes the 256^2 ping-pong kernel at D = 64 (the rotation from the stored bf16
 *   qkv in qk_rope_fwd's order: the same bits); otherwise owlk_gemm + owlk_qk_rope_fwd. */
int owlk_gemm_qk_rope(long M, long N, long K, const void* A, long lda, const void* W, long ldw, const float* bias,
                      void* qkv, long ldq, int H, int D, const float* cosb, const float* sinb, long ld_tab, long n_tab,
                      long tab_off, long tpos_div, void* out, long ldo, float* rstd, void* stream);
/* bytes of split-K workspace owlk_gemm uses for these arguments (0: no split) */
long owlk_gemm_splitk_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32, int epi,
                            float beta);
/* bytes of workspace for the deterministic form of a call: split-K partials, and with colsum != 0
 * the column-sum partials (fused or separate pass) */
long owlk_gemm_ws_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32, int epi,
                        float beta, int colsum);
/* leading bytes of that workspace that must be zero on entry (the decode plan's arrival counters,
 * OWLK_DECODE_COUNTER_BYTES; every launch leaves them zero); 0 when the plan keeps no state in ws */
long owlk_gemm_ws_counter_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32, int epi,
                                float beta);

/* ---- AdaLN modulate (modulation.py:7-26 AdaLN.forward after its fc; :46-55 cond_adaln):
 *   y[t] = bf16(bf16(bf16(rms_norm(x[t])) * bf16(1 + scale[t/tpf])) + shift[t/tpf]); rstd[t] fp32 */
int owlk_adaln_fwd(const void* x, long ldx, const void* scale, const void* shift, long ldm, long tpf,
                   long T, int d, void* y, long ldy, float* rstd, void* yact /* optional bf16(silu(y)),
                   FinalLayer attn.py:272-277 */, void* stream);
/* backward: dx = rms_norm' (dy * (1 + scale)) (+ dres); dscale[f] = sum_t dy*xn; dshift[f] = sum_t dy
 *   (fp32, or bf16 with mod_bf16 = 1: straight into a bf16 modulation-gradient matrix, row stride ldg) */
int owlk_adaln_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd,
                   const void* scale, long ldm, long tpf, long T, int d, const void* dres, long ldres,
                   void* dx, long lddx, void* dscale, void* dshift, long ldg,
                   const void* ypre /* optional: dy is d silu(ypre) */, int mod_bf16, void* stream);

/* ---- Gate backward (modulation.py:28-43 Gate / :57-63 cond_gate; forward is GEMM epi 2):
 *   dy = bf16(dout * g[t/tpf]); dg[f] = sum_t dout*y (row stride lddg; fp32, or bf16 with dg_bf16 = 1);
 *   dbias_frames[f] = sum_t dy (optional, fp32, row stride ldr) */
int owlk_gate_bwd(const void* dout, long ldo, const void* y, long ldy, const void* g, long ldg, long tpf,
                  long T, int d, void* dy, long lddy, void* dg, long lddg, int dg_bf16, float* dbias_frames,
                  long ldr, void* stream);
/* adaln_bwd then gate_bwd on the dx it forms, in one pass (the DiT block's MLP-branch AdaLN backward
 * feeding the attention branch's gate, modulation.py:28-55): dx as owlk_adaln_bwd (ypre none), then
 * dyg = bf16(dx * g[t/tpf]), dg[f] = sum_t dx*y, dbias_frames[f] = sum_t dyg (optional) -- bit for bit
 * the two calls, without reading dx back. */
int owlk_adaln_gate_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd,
                        const void* scale, long ldm, long tpf, long T, int d, const void* dres, long ldres,
                        void* dx, long lddx, void* dscale, void* dshift, long ldg, int mod_bf16,
                        const void* y, long ldy, const void* g, long ldgg, void* dyg, long lddyg, void* dg,
                        long lddg, int dg_bf16, float* dbias_frames, long ldr, void* stream);

/* ---- QK RMSNorm + RoPE (attn.py:83-89, rope.py:43-51): qkv rows [q(h d)|k(h d)|v(h d)] ->
 *   out rows [rope(bf16(rms(q)))|rope(bf16(rms(k)))], rotation pairs (2i, 2i+1) written to
 *   (i, D/2 + i); cos/sin fp32 tables [n_tab, D/2] (row stride ld_tab) at row
 *   tab_off + (tpos_div ? t % tpos_div : t).  Every row read must lie in the table (else returns 1:
 *   the reference's cos[offset:offset + n] slice comes out short and its rotation fails, rope.py:46-49). */
int owlk_qk_rope_fwd(const void* qkv, long ldq, long T, int H, int D, const float* cosb, const float* sinb,
                     long ld_tab, long n_tab, long tab_off, long tpos_div, void* out, long ldo, float* rstd,
                     void* stream);
/* decode form (attn.py:86-104 cache branch): q and k rotated as above, v copied, each into its own
 * destination (row stride ld*, batch stride s*; token t -> batch t / L, row t % L): k and v go
 * straight into the KV cache behind its window; no rstd */
int owlk_qk_rope_fwd_kv(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                        const float* sinb, long ld_tab, long n_tab, long tab_off, void* qo, long ldqo, long sqo,
                        void* ko, long ldko, long sko, void* vo, long ldvo, long svo, void* stream);
/* the same with the cache position on the device: state = {start, cached tokens, rope offset}
 * (int64), k / v written to rows start + cached + t of kbuf / vbuf ([B, cap, H D]), rope position
 * offset + t; one captured HIP graph then serves every frame of a growing cache.  A state whose rows
 * fall outside the cap buffer rows or the n_tab table rows is not followed: the kernel writes NaN q
 * rows and touches neither the cache nor the table. */
int owlk_qk_rope_fwd_kv_dev(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                            const float* sinb, long ld_tab, long n_tab, const long* state, void* qo, long ldqo,
                            long sqo, void* kbuf, long ldk, long skb, void* vbuf, long ldv, long svb, long cap,
                            void* stream);
int owlk_qk_rope_bwd(const void* dqk, long ldd, const void* qkv, long ldq, long T, int H, int D,
                     const float* cosb, const float* sinb, long ld_tab, long n_tab, long tab_off, long tpos_div,
                     const float* rstd, void* dqkv, long ldg, void* stream);
/* owlk_qk_rope_bwd with the column sums of its output fused: dbias[n] += sum_t bf16(dqkv[t, n]) for
 * n < 2 H D -- the q / k part of the qkv Linear's bias gradient (attn.py:90; torch's Linear backward
 * sums the bf16 output gradient over rows).  Per-token-block partials in ws (size from
 * owlk_qk_rope_bwd_ws_bytes; 0 = shape not supported by the fused form), added in a fixed order. */
long owlk_qk_rope_bwd_ws_bytes(long T, int H, int D);
int owlk_qk_rope_bwd_bias(const void* dqk, long ldd, const void* qkv, long ldq, long T, int H, int D,
                          const float* cosb, const float* sinb, long ld_tab, long n_tab, long tab_off, long tpos_div,
                          const float* rstd, void* dqkv, long ldg, float* dbias, void* ws, long ws_bytes,
                          void* stream);

/* ---- Frame-masked flash attention (replaces compiled flex_attention + create_block_mask,
 *   attn.py:13-16,24-62,106-109; mmattn.py:75).  q/k/v/o token-major rows (head h at column
 *   h*head_dim).  lse [B, H, Lq] fp32 in BASE 2: lse2[q] = log2 sum_k exp(scale * q.k) over the
 *   allowed keys (= the natural-log lse of flex_attention(..., return_lse=True) divided by ln 2;
 *   -inf for a row with no allowed key).  The backward entries take it in this form.  Mask: frame = (token + q_offset) / tpf for queries,
 *   token / tpf for keys; causal; |fq - fk| < window (window <= 0: unlimited); doc[b, fq] ==
 *   doc[b, fk].  Frame helper arrays (int32 [B, n_frames], batch stride fstride, may be NULL
 *   without docs): kv_lo (first visible kv frame), q_hi (last query frame seeing a kv frame),
 *   run_start (first frame of the contiguous same-doc run).
 * score_bound: 0, or a bound on |q.k| the caller guarantees for every pair (QK-RMSNorm'd q, k:
 *   sqrt(D) * sqrt(D) = D, attn.py:84, times 1 + a few bf16 ulps; scale * bound < 40); the
 *   softmax then needs no running row max: p = exp2(c s) directly (same result, no per-tile
 *   max / rescale; q is prescaled by c = scale * log2 e inside the kernel). */
int owlk_attn_fwd(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                  long ldv, long svb, void* o, long ldo, long sob, float* lse, long B, int H, long Lq,
                  long Lkv, int head_dim, float scale, float score_bound, long tpf, int window, int causal,
                  long q_offset,
                  const int* kv_lo, const int* q_hi, const int* run_start, const int* doc, long fstride,
                  void* stream);
/* Decode attention (attn.py:86-107 cache branch) with the cache position on the device: one frame
 * of Lq <= 64 queries per (batch, head), unmasked over [cache | Lnew new rows] of the cache
 * buffers kbuf / vbuf ([B, cap, H D]; the new rows written there first, owlk_qk_rope_fwd_kv_dev), or
 * over the last window_tokens of them (windowed layer; 0: all); state = {start, cached tokens, rope
 * offset} int64 on the device (rows past cap: NaN output, nothing read).  head_dim 64 or 128,
 * bounded softmax (score_bound > 0) only; lse base 2 as owlk_attn_fwd's. */
int owlk_attn_decode_fwd(const void* q, long ldq, long sqb, const void* kbuf, long ldk, long skb,
                         const void* vbuf, long ldv, long svb, void* o, long ldo, long sob, float* lse, long B,
                         int H, long Lq, int head_dim, float scale, float score_bound, const long* state,
                         long Lnew, long window_tokens, long cap, void* stream);
/* delta[b, h, t] = sum_d dO * O (fp32), the backward's row constant */
int owlk_attn_delta(const void* o, const void* dout, long ld, long B, long L, int H, int D, float* delta,
                    void* stream);
int owlk_attn_bwd(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                  long ldv, long svb, const void* dout, long ldo, long sob, const float* lse,
                  const float* delta, void* dq, long lddq, long sdqb, void* dk, long lddk, long sdkb,
                  void* dv, long lddv, long sdvb, long B, int H, long Lq, long Lkv, int head_dim,
                  float scale, long tpf, int window, int causal, const int* kv_lo, const int* q_hi,
                  const int* run_start, const int* doc, long fstride, void* stream);
/* the two phases of owlk_attn_bwd separately: dK/dV (key-owner sweep) and dQ (query-owner sweep) */
int owlk_attn_bwd_dkdv(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                       long ldv, long svb, const void* dout, long ldo, long sob, const float* lse,
                       const float* delta, void* dq, long lddq, long sdqb, void* dk, long lddk, long sdkb,
                       void* dv, long lddv, long sdvb, long B, int H, long Lq, long Lkv, int head_dim,
                       float scale, long tpf, int window, int causal, const int* kv_lo, const int* q_hi,
                       const int* run_start, const int* doc, long fstride, void* stream);
int owlk_attn_bwd_dq(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                     long ldv, long svb, const void* dout, long ldo, long sob, const float* lse,
                     const float* delta, void* dq, long lddq, long sdqb, void* dk, long lddk, long sdkb,
                     void* dv, long lddv, long sdvb, long B, int H, long Lq, long Lkv, int head_dim,
                     float scale, long tpf, int window, int causal, const int* kv_lo, const int* q_hi,
                     const int* run_start, const int* doc, long fstride, void* stream);

/* Single-pass backward (head_dim 64, Lq == Lkv == L; frame masks windowed or not, and causal masks of packed
 * documents given as kv_lo / q_hi alone, every document one run of frames -- run_start / doc must be
 * null, as owlk_attn_bwd's runs form): the same
 * outputs as owlk_attn_bwd from ONE kernel -- the compiled flex_attention backward of
 * attn.py:13-16,106-109 is likewise one pass.  Each 256-key block forms S and dP once and adds its
 * dQ part to a per-query-tile fp32 sum in the workspace in key-block order (ordered hand-off, no
 * float atomics: dQ is bitwise reproducible).  ws: caller-owned, >= owlk_attn_bwd_fused_ws_bytes,
 * 256-B aligned; the entry zeroes its header / flags itself (one memset on the stream).  variant:
 * 0 = write-through (sc1) sums, any workgroup placement; bit 0 = a chain's sums kept in one XCD's
 * L2 (plain stores, per-XCD queues; taken only on a device of 8 XCCs, hipDeviceAttributeNumberOfXccs,
 * else the call runs write-through); bits 2-5 = chains of an XCD queue swept at a time (0 = all of
 * them interleaved; 1 gives each chain every workgroup of its XCD, so its sums and Q / dO tiles are
 * re-read fewer times); bit 1 = test mode: every contributor adds 1.0
 * instead of its dQ part and the last one keeps the fp32 sum in ws (dQ not written); bit 6 = test mode:
 * chain 0's key block 1 times out on its hand-off waits.  A hand-off wait that times out (2 s; never
 * expected) sets ws int32 word 8 to 1 and makes the tile's dQ NaN (every later part of the sum
 * carries it, so the stored rows are NaN); after one timeout every later wait gives up at once.  In
 * the XCD-local form a queue left undrained (no workgroup on its XCD) sets word 8 to 2 and its
 * chains' dQ, dK and dV rows are written NaN.  No wrong gradient leaves the call looking valid. */
long owlk_attn_bwd_fused_ws_bytes(long B, int H, long L, int head_dim);
int owlk_attn_bwd_fused(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                        long ldv, long svb, const void* dout, long ldo, long sob, const float* lse,
                        const float* delta, void* dq, long lddq, long sdqb, void* dk, long lddk, long sdkb,
                        void* dv, long lddv, long sdvb, long B, int H, long L, int head_dim, float scale,
                        long tpf, int window, int causal, const int* kv_lo, const int* q_hi,
                        const int* run_start, const int* doc, long fstride, void* ws, long ws_bytes,
                        int variant, void* stream);
/* CUs the persistent single-pass backward leaves free for kernels on other streams (the gradient
 * all-reduce of the synchronising micro-step, utils/grad_reducer.py): its grid becomes (CUs - cus)
 * workgroups per CU-slot, at least one per XCD.  Process-wide; 0 (default) = every CU.  Replaces
 * nothing in the reference: DDP's bucketed all-reduce overlaps backward there (rft_trainer.py:95-99),
 * and on MI355X a persistent grid on every CU would hold a bucket's collective until it ends. */
int owlk_set_cu_reserve(int cus);

/* ---- Flow-matching noise + patchify (gamerft.py:92-95,107-108,52): x, z [BN, C, P] bf16,
 *   ts_raw [BN] fp32 (bf16-valued randn) -> xt, tgt token-major [BN*P, C]; ts_out = bf16 sigmoid */
int owlk_flow_noise(const void* x, const void* z, const float* ts_raw, int C, int P, long BN, void* xt,
                    void* tgt, float* ts_out, void* stream);
/* token-major [BN*P, C] -> [BN, C, P] (gamerft.py:58) */
int owlk_unpatchify(const void* tok, int C, int P, long BN, void* out, void* stream);
/* out = bf16(x + bf16(g[t / tpf] * y)), [T, d] bf16 rows: the GATE_RESID GEMM epilogue's output
 * recomputed bit for bit from its kept inputs (residual x, gated branch y, per-frame gate g) */
int owlk_gate_resid(const void* x, long ldx, const void* y, long ldy, const void* g, long ldg, long tpf, long T,
                    int d, void* out, long ldo, void* stream);
/* MSE (gamerft.py:111): partial[block] = sum (pred - tgt)^2; dpred (optional) = bf16(gscale * (pred - tgt));
 * loss (optional, fp32 scalar) = (float)(double sum of the partials in block order) / n */
int owlk_mse(const void* pred, const void* tgt, long n, float gscale, void* dpred, float* partial,
             int nblocks, float* loss, void* stream);
/* its backward: dpred = bf16((gscale * (pred - tgt)) * gout[0]) (gout NULL: 1), gscale = 2 / n for the mean */
int owlk_mse_grad(const void* pred, const void* tgt, long n, float gscale, const float* gout, void* dpred,
                  void* stream);
/* out[n] += sum_r x[r, n] (bias gradients); x bf16 (x_f32 = 0) or fp32.  With ws (>=
 * owlk_colsum_ws_bytes(R, N) bytes, 16-B aligned) row splits store partial rows that one pass adds
 * in order (bitwise deterministic); without it the splits combine by fp32 atomics. */
long owlk_colsum_ws_bytes(long R, long N);
int owlk_colsum(const void* x, int x_f32, long R, long N, long ld, float* out, void* ws, long ws_bytes,
                void* stream);
/* owlk_colsum over frame-strided rows (row r at (r / OWLK_FRAME_ROWS) * fs + (r % OWLK_FRAME_ROWS) * ld;
 * fs = 0: plain): the MMDiT video qkv bias gradient summed in place over the joint rows */
int owlk_colsum_frames(const void* x, int x_f32, long R, long N, long ld, long fs, float* out, void* ws,
                       long ws_bytes, void* stream);

/* ---- Newton-Schulz (muon.py:11-38) helpers: X /= (||X||_F + eps) per batch item, bf16.
 * Norms are reduced without atomics: sum-of-squares passes write OWLK_NORM_PARTS partial sums per
 * matrix and the scale pass adds them in fixed order (bitwise reproducible).
 * work: fp32 [batch, OWLK_NORM_PARTS] scratch (fully written; no zeroing needed). */
#define OWLK_NORM_PARTS 256
int owlk_ns_normalize(const void* g, int g_f32, long rows, long cols, long batch, int transpose, void* x,
                      float* work, void* stream);
/* the scale pass of owlk_ns_normalize alone, given sumsq [batch, OWLK_NORM_PARTS] partials of
 * sum(bf16(g)^2) per matrix (what owlk_muon_momentum writes) */
int owlk_ns_scale(const void* g, int g_f32, long rows, long cols, long batch, int transpose, void* x,
                  const float* sumsq, void* stream);
/* The quintic iterations of muon.py:30-34, in place on a normalised bf16 X [batch, m, k]
 *   (contiguous, m <= k, both multiples of 8), in the eager reference's rounding order:
 *   A = X X^T; B = bf16(b A) + bf16(bf16(c A) @ A); X = bf16(a X) + bf16(B @ X).
 *   ws: caller-owned, >= owlk_ns_iterate_ws_bytes(batch, m, k) bytes, 16-B aligned. */
long owlk_ns_iterate_ws_bytes(long batch, long m, long k);
int owlk_ns_iterate(void* x, long batch, long m, long k, int steps, float a, float b, float c, void* ws,
                    long ws_bytes, void* stream);
/* zeropower_via_newtonschulz5 (muon.py:11-38) as one entry: g [batch, rows, cols] fp32 (g_f32 = 1)
 *   or bf16 -> out bf16 [batch, rows, cols]; transposes when rows > cols and zero-pads dims that
 *   are not multiples of 8 internally.  Reference coefficients (a, b, c) = (3.4445, -4.7750, 2.0315).
 *   ws: caller-owned, >= owlk_newton_schulz_ws_bytes(batch, rows, cols) bytes, 16-B aligned. */
long owlk_newton_schulz_ws_bytes(long batch, long rows, long cols);
int owlk_newton_schulz_bf16(const void* g, int g_f32, long batch, long rows, long cols, int steps, float a,
                            float b, float c, void* out, void* ws, long ws_bytes, void* stream);

/* ---- per-frame conditioning (cond.hip; GameRFTCore.cond gamerft.py:39-48, embeddings.py:30-184,
 *   the silu(cond) of every modulation fc modulation.py:13,32).  Each op rounds as the reference's
 *   torch op does: to bf16 when its input is bf16 (*_f32 = 0), not at all when fp32 (*_f32 = 1);
 *   every output is the bf16 operand autocast hands the next Linear.
 * owlk_cond_embed: R rows ->
 *   ts_in [R, 2 ht] = [sin e | cos e], e = (ts * tmult) * tfreq[i] (SinCosEmbed; tfreq fp32 [ht]);
 *   mouse_in [R, 4 hm]: [:, :2 hm] = angle_proj(cos, sin of the symlog polar angle) with wang fp32 [2 hm, 2]
 *     (bf16 operands, fp32 sum), [:, 2 hm:] = SinCos(|symlog mouse|) (mfreq fp32 [hm]); mouse row stride ldm;
 *     ang [R, 2] bf16 = (cos, sin), kept for the angle_proj weight gradient;
 *   btn_in [R, nbp] = 2 b - 1 (columns nb .. nbp zero).  ts / mouse / btn may each be NULL. */
int owlk_cond_embed(const void* ts, int ts_f32, const float* tfreq, int ht, float tmult, void* ts_in, long ldt,
                    const void* mouse, int mouse_f32, long ldm, const float* mfreq, int hm, float mmult,
                    const float* wang, void* mouse_in, long ldmi, void* ang, const void* btn, int btn_f32, long ldb,
                    int nb, int nbp, void* btn_in, long ldbi, long R, void* stream);
/* cond = bf16(t + (hc[row / rows_per] ? bf16(m + b) : 0)) (m, b NULL: cond = t; hc: bool per sample,
 * NULL: all true); s = bf16(silu(cond)); cond may be NULL (not kept).  Contiguous [R, d] bf16. */
int owlk_cond_silu_fwd(const void* t, const void* m, const void* b, const void* hc, long rows_per, long R, int d,
                       void* cond, void* s, void* stream);
/* backward: ds [R, d] (fp32: all consumers of s, summed; or bf16 with ds_bf16 = 1) ->
 * dcond = bf16(bf16(ds) silu'(cond)) (cond NULL: dcond = ds, the gradient of cond itself);
 * dctrl = hc ? dcond : 0.  dcond / dctrl optional. */
int owlk_cond_silu_bwd(const void* ds, int ds_bf16, const void* cond, const void* hc, long rows_per, long R, int d,
                       void* dcond, void* dctrl, void* stream);
/* dw[n, k] (row stride ldw, fp32) = beta * dw + sum_r dy[r, n] * x[r, k] for k < K <= 16, rows in a
 * fixed order: the weight gradients of the embeddings' K = 2 / 11 input layers (angle_proj,
 * button fc1), which the 8-aligned GEMM does not tile */
int owlk_small_k_wgrad(const void* dy, long lddy, const void* x, long ldx, long R, long N, int K, float* dw,
                       long ldw, float beta, void* stream);

/* ---- fused Muon passes (optim.hip; replace muon.py:66-84's torch elementwise ops) ----
 * owlk_muon_momentum: for each of `count` fp32 matrices of n elements (host array of device
 *   pointers g[i], buf[i]): buf = lerp(buf, g, 1 - momentum); g' = nesterov ? lerp(g, buf, momentum)
 *   : buf (muon.py:67-73).  g' goes to stack[i*n ...] (fp32, the batched NS input) or, with
 *   stack == NULL, back into g (the reference's in-place update).  sumsq: fp32 [count,
 *   OWLK_NORM_PARTS], written with the partial sums of sum(bf16(g')^2) (NULL skips), the
 *   Frobenius-norm input of owlk_ns_scale (muon.py:24-26).
 * owlk_muon_apply: p[i] = p[i] * decay - alpha * u[i] (muon.py:80-84: decay = 1 - lr*wd,
 *   alpha = lr * max(1, rows/cols)^0.5); u bf16 [count, rows, cols], or [count, cols, rows] with
 *   transpose = 1 (the NS iterate before its transpose back). */
int owlk_muon_momentum(int count, float* const* g, float* const* buf, long n, float momentum, int nesterov,
                       float* stack, float* sumsq, void* stream);
int owlk_muon_apply(int count, float* const* p, const void* u, long rows, long cols, int transpose, float decay,
                    float alpha, void* stream);
/* AdamW step over `count` fp32 tensors of n[i] elements (host arrays of device pointers), in
 * torch.optim.AdamW's order (replaces the foreach AdamW of muon.py:143-146 / rft_trainer.py):
 * p *= 1 - lr*wd; m = lerp(m, g, 1 - beta1); v = v*beta2 + (1 - beta2) g^2;
 * p += step_size * m / (sqrt(v) / bc2_sqrt + eps), step_size = -lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t). */
int owlk_adamw(int count, float* const* p, const float* const* g, float* const* m, float* const* v, const long* n,
               float lr, float beta1, float beta2, float weight_decay, float eps, float step_size, float bc2_sqrt,
               void* stream);
/* EMA of the weights (rft_trainer.py:105, ema_pytorch): shadow[i] = lerp(shadow[i], p[i], weight) over
 * `count` fp32 tensors of n[i] elements, torch's lerp formula (weight = 1 - decay). */
int owlk_ema(int count, float* const* shadow, const float* const* p, const long* n, float weight, void* stream);

/* ---- MMDiT plumbing (frames.hip) ----
 * owlk_frame_mux replaces the per-frame concat / split of mmattn.py:54-60 and :77-80: frame f of
 * the joint sequence is [n0 rows of a (video) | n1 rows of b (audio)].  dir 0: a, b -> joint;
 * dir 1: joint -> a, b.  `frames` counts frames over the whole batch; cols % 8 == 0 (bf16). */
int owlk_frame_mux(int dir, long frames, int n0, int n1, int cols, void* a, long lda, void* b, long ldb,
                   void* joint, long ldj, void* stream);
/* F.layer_norm(x, (d,)) without affine, eps 1e-5, fp32 math, bf16 in/out (normalization.py:6-7,
 * used on the MMDiT video head, gamerft_audio.py:89); mean / rstd fp32 [T] saved for backward */
int owlk_layernorm_fwd(const void* x, long ldx, long T, int d, void* y, long ldy, float* mean, float* rstd,
                       void* stream);
int owlk_layernorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* mean, const float* rstd,
                       long T, int d, void* dx, long lddx, void* stream);

#ifdef __cplusplus
}
#endif
#endif
