// Host-side launchers of the drtc_amd HIP kernels.  Every launcher enqueues
// on the caller's stream only (no allocation, no synchronisation) so the
// whole decode step can be captured into a hipGraph.  Return value: 0 on
// success, a negative code on an unsupported shape, else a hipError_t.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <vector>

namespace drtc {

int launch_rmsnorm(void* out, void* residual, const void* x, const void* w,
                   int rows, int H, float eps, int x_stride, int out_stride,
                   int res_stride, bool gemma, hipStream_t st);

int launch_act_glu(void* out, const void* gu, int64_t T, int I, int gu_stride,
                   int act, hipStream_t st);

void set_rope_variant(int v);
int launch_rope_kv(void* qkv, int T, int qkv_stride, const int* positions,
                   const int64_t* slots, const float* cos_sin, int Hq, int Hkv,
                   int D, void* k_cache, void* v_cache, int block_size, int write_v,
                   hipStream_t st);

int launch_kv_write_v(void* v_cache, const void* qkv, int qkv_stride, const int* seg_tok,
                      const int* seg_len, const int* seg_blk, int nseg, int Hq, int Hkv,
                      int D, int block_size, hipStream_t st);

int launch_paged_decode_rope(void* out, float* part_o, float* part_ml, const void* q,
                             int q_stride, void* k_cache, void* v_cache,
                             const int* block_tables, int bt_stride, const int* context_lens,
                             int B, int Hq, int Hkv, int D, float scale, int max_parts,
                             int blocks_per_part, const int* positions, const int64_t* slots,
                             const float* cos_sin, int max_wgs, hipStream_t st);
int launch_paged_decode(void* out, float* part_o, float* part_ml, int* counters, const void* q,
                        int q_stride, const void* k_cache, const void* v_cache,
                        const int* block_tables, int bt_stride,
                        const int* context_lens, int B, int Hq, int Hkv, int D,
                        float scale, int max_parts, int blocks_per_part, int variant,
                        hipStream_t st);

int launch_prefill_attn(void* out, int out_stride, const void* qkv,
                        int qkv_stride, int Hq, int Hkv, int D,
                        const int* cu_seqlens, const int* tile_seq,
                        const int* tile_q0, int ntiles, float scale, int causal, int persist,
                        hipStream_t st);

int launch_sample(int* out_tokens, const void* logits, int B, int V, int ld,
                  const float* temperature, const int* top_k, const float* top_p,
                  uint64_t seed, const int64_t* step, hipStream_t st);

// variant 0 / 1 / 2: the moe.hip grouped GEMMs; 3: gemm_xd grouped mode with xd forms gu_form
// (gated gate_up) / dn_form (down), 0 = by rows per expert; slab / counters: the split-K
// workspace of the gemm_xd forms (may be null: no split-K); 4: rows gathered into expert order,
// then gemm_w4's grouped persistent form (prefill-sized rows per expert); -1: by rows per
// expert
int launch_moe(void* out, const void* x, const void* router_logits, const void* w_gu,
               const void* w_dn, int T, int H, int I, int E, int k, int e_off, int e_local,
               int act, void* workspace, int64_t ws_bytes, int variant, int gu_form, int dn_form,
               void* slab, int64_t slab_bytes, int* counters, int n_counters, int logit_ts,
               int logit_es, hipStream_t st);
int64_t moe_workspace_bytes(int T, int H, int I, int e_local, int k);
void moe_set_w4_group_m(int gu, int dn);  // variant 4 tile-order row groups (A/B knob)
// Expert-parallel dispatch / combine with a static per-destination capacity (moe_ep.hip).
int launch_ep_plan(const int* topi, int P, int e_local, int world, int cap, int* dst_row,
                   int* send_pair, int* send_e, int* overflow, hipStream_t st);
int launch_ep_gather(void* send_x, const void* x, const int* send_pair, int rows, int k, int H,
                     int ldx, hipStream_t st);
int launch_ep_combine(void* out, const void* back, const int* dst_row, const float* w, int T,
                      int k, int H, hipStream_t st);

// One-shot P2P all-reduce over IPC-mapped staging buffers (allreduce.hip).
struct ArPeers {
  char* base[8];
};
int64_t custom_ar_buffer_bytes(int64_t stage_elems);
int launch_custom_allreduce(void* out, const void* in, int64_t n, const ArPeers& peers, int rank,
                            int world, int64_t stage_elems, int two_shot, hipStream_t st);
int ar_alloc(void** p, int64_t bytes);
int ar_free(void* p);
int ar_ipc_get(void* p, char* handle);  // 64-byte handle
int ar_ipc_open(const char* handle, void** p);
int ar_ipc_close(void* p);
int ar_error(void* base);
// One-shot all-reduce + residual add + RMSNorm (decode sublayer epilogue under TP).
int launch_custom_ar_rmsnorm(void* normed, void* residual, const void* in, const void* w,
                             int rows, int H, float eps, int gemma, const ArPeers& peers,
                             int rank, int world, int64_t stage_elems, hipStream_t st);
int ar_set_epoch(void* base, uint64_t epoch);

// Tuned hipBLASLt projection GEMM y[M,N] = x[M,K] @ W[N,K]^T + beta * y, bf16 (gemm_lt.cpp).
int lt_version();
int lt_gemm(void* y, const void* x, const void* w, int64_t M, int64_t N, int64_t K, int64_t ldx,
            int64_t ldy, float beta, hipStream_t st);
int lt_set_algo(int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldy, int algo_index);
// (solution index, us per call) pairs; index -1 = hipBLASLt's heuristic pick
std::vector<std::pair<int, float>> lt_tune(void* y, const void* x, const void* w, int64_t M,
                                           int64_t N, int64_t K, int64_t ldx, int64_t ldy,
                                           int iters, int max_candidates, hipStream_t st);

// Skinny projection GEMM for decode batches M <= 16 (gemv.hip): y[M,N] = x[M,K] @ W[N,K]^T.
// variant 0 = by shape; returns -1 for a shape the chosen form does not cover.
int launch_skinny_gemm(void* y, const void* x, const void* w, int M, int N, int K, int ldx,
                       int ldy, int variant, hipStream_t st);

// Gated activation fused into the skinny dot2 GEMM (gemv.hip): y = (act(gu[:, :K]) * gu[:, K:2K]) @ W^T,
// gu row stride ldx; M <= 2, K % 512 == 0, act 0 = SiLU, 1 = tanh-GELU.
int launch_skinny_glu_gemm(void* y, const void* gu, const void* w, int M, int N, int K, int ldx,
                           int ldy, int act, hipStream_t st);
// RMSNorm (+ residual add) fused into the skinny dot2 GEMM (gemv.hip): y = norm(x [+ res]) @ W^T,
// h_out = x + res (written when res is given); M <= 4, K % 2048 == 0.
int launch_skinny_norm_gemm(void* y, void* h_out, const void* x, const void* res, const void* nw,
                            const void* w, int M, int N, int K, int ldx, int ldr, int ldh,
                            int ldy, float eps, bool gemma, hipStream_t st);

// 4-wave hand-scheduled GEMM (gemm_w4.hip): c[M,N] = epi(a[M,K] . b[N,K]^T); epi 0 store,
// 1 + r (residual, may alias c), 2/3 SiLU/GELU gated (b rows [0,up_off) gate, [up_off, 2 up_off)
// up, N = up_off).  v = schedule bits (0 per-tile, 2 temporal stores, 8 persistent, 24
// persistent + per-XCD K rotation); splitk > 1 (per-tile form) needs slab + counters (zeroed
// once): 256 KiB of slab per tile and slice.
void w4_set_krot(int k);
void w4_set_grouped_rot(int r);
int w4_krot();
int launch_gemm_w4(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldr, int epi, int up_off, int splitk,
                   int group_m, void* slab, int64_t slab_bytes, int* counters, int n_counters,
                   int v, hipStream_t st);
// Grouped persistent form: rows [grp[g], grp[g + 1]) of a / c (grp: n_grp + 1 row offsets in
// DEVICE memory) times weight b + g * b_grp; epi 0 store or 2/3 gated; max_rows >= grp[n_grp]
// sizes the grid.  ksplit > 1 (store only): K cut into ksplit slices, slice s written as bf16
// partial products to c + s * c_split elements.
int launch_gemm_w4_grouped(void* c, const void* a, const void* b, const int* grp, int n_grp,
                           int max_rows, int N, int K, int lda, int ldb, int ldc, int64_t b_grp,
                           int epi, int up_off, int group_m, int ksplit, int64_t c_split,
                           hipStream_t st);
int64_t gemm_w4_workspace_bytes(int64_t M, int64_t N, int splitk);
int configure_gemm_w4();


// XCD-partitioned decode GEMM (gemm_xd.hip): c[M,N] = epi(a[M,K] . b[N,K]^T); epi 0 store, 1 + r
// (residual, may alias c), 2 / 3 SiLU / GELU gating of b = [gate; up] (2 N rows); 128 mt x 32 nf
// tiles ((mt, nf) in (1, 2/4/6), (2, 4/6); gated: 16 nf output columns, nf even), K split over
// splitk = 1..8 slices (splitk > 1: slab + counters zeroed once, gemm_xd_workspace_bytes), one
// workgroup per tile and slice; N % tile columns == 0, K % 64 == 0, K / 64 / splitk > ring.
int launch_gemm_xd(void* c, const void* a, const void* b, const void* r, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldr, int epi, int mt, int nf, int splitk,
                   void* slab, int64_t slab_bytes, int* counters, int n_counters,
                   hipStream_t st);
int64_t gemm_xd_workspace_bytes(int M, int N, int mt, int nf, int splitk, int glu);
// Grouped (mixture-of-experts) gemm_xd: row tile i of C / A is entry i < *n_tiles of a device
// tile table (rows [tile_row0[i], + tile_rows[i]), expert tile_expert[i]: weights b +
// expert * b_stride elements); A rows gathered through a_index when given (a_rows = rows of A
// then).  Forms (mt, nf) in (1, 4), (2, 4), (2, 8), + 16 in mt for non-temporal weight loads;
// epi 0 store, 2 / 3 SiLU / GELU gated.  Grid: max_tiles x column tiles x splitk workgroups.
int launch_gemm_xd_grouped(void* c, const void* a, const void* b, int a_rows, int N, int K,
                           int lda, int ldb, int ldc, int epi, int mt, int nf, int splitk,
                           int max_tiles, const int* tile_row0, const int* tile_rows,
                           const int* tile_expert, const int* n_tiles, const int* a_index,
                           int64_t b_stride, void* slab, int64_t slab_bytes, int* counters,
                           int n_counters, hipStream_t st);
int configure_gemm_xd();
// Split-K fault handling shared by gemm_xd and gemm_w4: a combine whose poll for the other
// slices exceeds the spin limit stores 1 into the workspace's LAST counter (n_counters - 1,
// outside every launch's ticket range) and leaves the counters un-armed; the host reads that
// word (ops.gemm.check_splitk_fault), zeroes the counters and raises.  The limit is a process
// setting (default 1 << 24 polls); < 0 forces every combine to fault (tests only).
int splitk_spin_limit();
void set_splitk_spin_limit(int limit);

// Raise the dynamic-LDS ceiling of the kernels that need > 64 KiB (head_dim
// 256).  Called once at import, before any graph capture.
int configure_kernels();
int configure_decode();
int configure_prefill();
// medium-M decode GEMM (gemm_midm.hip)
int64_t midm_slab_bytes(int M, int N, int S);
int launch_midm_gemm(void* y, const void* x, const void* w, const void* res, int M, int N,
                     int K, int ldx, int ldy, int ldr, int epi, int S, void* slab,
                     int64_t slab_bytes, hipStream_t st);
int configure_moe();

}  // namespace drtc
