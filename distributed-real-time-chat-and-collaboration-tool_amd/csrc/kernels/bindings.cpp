// pybind11 module `_hipk`: thin bindings over the HIP launchers.
//
// Tensors cross the boundary as raw device addresses (Python passes
// `tensor.data_ptr()`) and the stream as `torch.cuda.current_stream()
// .cuda_stream`; shape/dtype validation happens in the Python op wrappers
// (drtc_amd/ops), which also check every launcher's return code.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <vector>

#include "launchers.h"

namespace py = pybind11;
using u64 = std::uintptr_t;

template <class T>
static T* P(u64 p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(u64 s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_hipk, m) {
  m.doc() = "drtc_amd CDNA4 (gfx950) HIP kernels";
  m.def("configure", []() { return drtc::configure_kernels(); });
  m.def("rmsnorm",
        [](u64 out, u64 residual, u64 x, u64 w, int rows, int H, float eps,
           int x_stride, int out_stride, int res_stride, bool gemma, u64 st) {
          return drtc::launch_rmsnorm(P<void>(out), P<void>(residual), P<void>(x),
                                      P<void>(w), rows, H, eps, x_stride,
                                      out_stride, res_stride, gemma, S(st));
        });
  m.def("act_glu", [](u64 out, u64 gu, int64_t T, int I, int gu_stride, int act,
                      u64 st) {
    return drtc::launch_act_glu(P<void>(out), P<void>(gu), T, I, gu_stride, act, S(st));
  });
  m.def("rope_kv", [](u64 qkv, int T, int qkv_stride, u64 positions, u64 slots,
                      u64 cos_sin, int Hq, int Hkv, int D, u64 k_cache,
                      u64 v_cache, int block_size, int write_v, u64 st) {
    return drtc::launch_rope_kv(P<void>(qkv), T, qkv_stride, P<const int>(positions),
                                P<const int64_t>(slots), P<const float>(cos_sin), Hq,
                                Hkv, D, P<void>(k_cache), P<void>(v_cache),
                                block_size, write_v, S(st));
  });
  m.def("set_rope_variant", [](int v) { drtc::set_rope_variant(v); });
  m.def("w4_set_krot", [](int k) { drtc::w4_set_krot(k); });
  m.def("w4_krot", []() { return drtc::w4_krot(); });
  m.def("w4_set_grouped_rot", [](int r) { drtc::w4_set_grouped_rot(r); });
  m.def("kv_write_v", [](u64 v_cache, u64 qkv, int qkv_stride, u64 seg_tok, u64 seg_len,
                         u64 seg_blk, int nseg, int Hq, int Hkv, int D, int block_size,
                         u64 st) {
    return drtc::launch_kv_write_v(P<void>(v_cache), P<const void>(qkv), qkv_stride,
                                   P<const int>(seg_tok), P<const int>(seg_len),
                                   P<const int>(seg_blk), nseg, Hq, Hkv, D, block_size, S(st));
  });
  m.def("paged_decode",
        [](u64 out, u64 part_o, u64 part_ml, u64 counters, u64 q, int q_stride, u64 k_cache,
           u64 v_cache, u64 block_tables, int bt_stride, u64 context_lens, int B,
           int Hq, int Hkv, int D, float scale, int max_parts,
           int blocks_per_part, int variant, u64 st) {
          return drtc::launch_paged_decode(
              P<void>(out), P<float>(part_o), P<float>(part_ml), P<int>(counters), P<const void>(q),
              q_stride, P<const void>(k_cache), P<const void>(v_cache),
              P<const int>(block_tables), bt_stride, P<const int>(context_lens), B,
              Hq, Hkv, D, scale, max_parts, blocks_per_part, variant, S(st));
        });
  m.def("paged_decode_rope",
        [](u64 out, u64 part_o, u64 part_ml, u64 qkv, int q_stride, u64 k_cache, u64 v_cache,
           u64 block_tables, int bt_stride, u64 context_lens, int B, int Hq, int Hkv, int D,
           float scale, int max_parts, int blocks_per_part, u64 positions, u64 slots,
           u64 cos_sin, int max_wgs, u64 st) {
          return drtc::launch_paged_decode_rope(
              P<void>(out), P<float>(part_o), P<float>(part_ml), P<const void>(qkv), q_stride,
              P<void>(k_cache), P<void>(v_cache), P<const int>(block_tables), bt_stride,
              P<const int>(context_lens), B, Hq, Hkv, D, scale, max_parts, blocks_per_part,
              P<const int>(positions), P<const int64_t>(slots), P<const float>(cos_sin), max_wgs,
              S(st));
        });
  m.def("prefill_attn",
        [](u64 out, int out_stride, u64 qkv, int qkv_stride, int Hq, int Hkv,
           int D, u64 cu_seqlens, u64 tile_seq, u64 tile_q0, int ntiles,
           float scale, int causal, int persist, u64 st) {
          return drtc::launch_prefill_attn(
              P<void>(out), out_stride, P<const void>(qkv), qkv_stride, Hq, Hkv, D,
              P<const int>(cu_seqlens), P<const int>(tile_seq),
              P<const int>(tile_q0), ntiles, scale, causal, persist, S(st));
        });
  m.def("moe", [](u64 out, u64 x, u64 logits, u64 w_gu, u64 w_dn, int T, int H, int I, int E,
                  int k, int e_off, int e_local, int act, u64 ws, int64_t ws_bytes, int variant,
                  int gu_form, int dn_form, u64 slab, int64_t slab_bytes, u64 counters,
                  int n_counters, int logit_ts, int logit_es, u64 st) {
    return drtc::launch_moe(P<void>(out), P<const void>(x), P<const void>(logits),
                            P<const void>(w_gu), P<const void>(w_dn), T, H, I, E, k, e_off,
                            e_local, act, P<void>(ws), ws_bytes, variant, gu_form, dn_form,
                            P<void>(slab), slab_bytes, P<int>(counters), n_counters, logit_ts,
                            logit_es, S(st));
  });
  // gemm_w4 (ops.gemm.mfma_gemm): variant 7 + schedule bits (7 per-tile, 9 temporal stores,
  // 15 persistent, 31 persistent with the per-XCD K rotation)
  m.def("gemm", [](u64 c, u64 a, u64 b, u64 r, int M, int N, int K, int lda, int ldb, int ldc,
                   int ldr, int epi, int up_off, int variant, int splitk, int group_m, u64 slab,
                   int64_t slab_bytes, u64 counters, int n_counters, u64 st) {
    if (variant < 7) return -1;
    return drtc::launch_gemm_w4(P<void>(c), P<const void>(a), P<const void>(b), P<const void>(r),
                                M, N, K, lda, ldb, ldc, ldr, epi, up_off, splitk, group_m,
                                P<void>(slab), slab_bytes, P<int>(counters), n_counters,
                                variant - 7, S(st));
  });
  // gemm_w4 grouped persistent form (ops.gemm.mfma_gemm_grouped): per-group weights, device
  // row offsets
  m.def("gemm_grouped", [](u64 c, u64 a, u64 b, u64 grp, int n_grp, int max_rows, int N, int K,
                           int lda, int ldb, int ldc, int64_t b_grp, int epi, int up_off,
                           int group_m, int ksplit, int64_t c_split, u64 st) {
    return drtc::launch_gemm_w4_grouped(P<void>(c), P<const void>(a), P<const void>(b),
                                        P<const int>(grp), n_grp, max_rows, N, K, lda, ldb, ldc,
                                        b_grp, epi, up_off, group_m, ksplit, c_split, S(st));
  });
  // gemm_xd (ops.gemm.xd_gemm): decode-shaped tiles, XCD-partitioned order, split-K 1..8
  m.def("gemm_xd", [](u64 c, u64 a, u64 b, u64 r, int M, int N, int K, int lda, int ldb, int ldc,
                      int ldr, int epi, int mt, int nf, int splitk, u64 slab, int64_t slab_bytes,
                      u64 counters, int n_counters, u64 st) {
    return drtc::launch_gemm_xd(P<void>(c), P<const void>(a), P<const void>(b), P<const void>(r),
                                M, N, K, lda, ldb, ldc, ldr, epi, mt, nf, splitk, P<void>(slab),
                                slab_bytes, P<int>(counters), n_counters, S(st));
  });
  m.def("gemm_xd_workspace_bytes", &drtc::gemm_xd_workspace_bytes);
  m.def("splitk_spin_limit", &drtc::splitk_spin_limit);
  m.def("set_splitk_spin_limit", &drtc::set_splitk_spin_limit);
  m.def("gemm_workspace_bytes", &drtc::gemm_w4_workspace_bytes);
  m.def("moe_workspace_bytes", &drtc::moe_workspace_bytes);
  m.def("moe_set_w4_group_m", [](int gu, int dn) { drtc::moe_set_w4_group_m(gu, dn); });
  m.def("ep_plan", [](u64 topi, int npairs, int e_local, int world, int cap, u64 dst_row,
                      u64 send_pair, u64 send_e, u64 overflow, u64 st) {
    return drtc::launch_ep_plan(P<const int>(topi), npairs, e_local, world, cap, P<int>(dst_row),
                                P<int>(send_pair), P<int>(send_e), P<int>(overflow), S(st));
  });
  m.def("ep_gather", [](u64 send_x, u64 x, u64 send_pair, int rows, int k, int H, int ldx, u64 st) {
    return drtc::launch_ep_gather(P<void>(send_x), P<const void>(x), P<const int>(send_pair), rows,
                                  k, H, ldx, S(st));
  });
  m.def("ep_combine", [](u64 out, u64 back, u64 dst_row, u64 w, int T, int k, int H, u64 st) {
    return drtc::launch_ep_combine(P<void>(out), P<const void>(back), P<const int>(dst_row),
                                   P<const float>(w), T, k, H, S(st));
  });
  m.def("custom_ar_buffer_bytes", &drtc::custom_ar_buffer_bytes);
  m.def("custom_allreduce", [](u64 out, u64 in, int64_t n, const std::vector<u64>& bases, int rank,
                               int64_t stage_elems, int two_shot, u64 st) {
    drtc::ArPeers p{};
    if (bases.size() > 8) return -1;
    for (size_t i = 0; i < bases.size(); ++i) p.base[i] = P<char>(bases[i]);
    return drtc::launch_custom_allreduce(P<void>(out), P<const void>(in), n, p, rank,
                                         (int)bases.size(), stage_elems, two_shot, S(st));
  });
  m.def("custom_ar_rmsnorm", [](u64 normed, u64 residual, u64 in, u64 w, int rows, int H,
                                float eps, bool gemma, const std::vector<u64>& bases, int rank,
                                int64_t stage_elems, u64 st) {
    drtc::ArPeers p{};
    if (bases.size() > 8) return -1;
    for (size_t i = 0; i < bases.size(); ++i) p.base[i] = P<char>(bases[i]);
    return drtc::launch_custom_ar_rmsnorm(P<void>(normed), P<void>(residual), P<const void>(in),
                                          P<const void>(w), rows, H, eps, gemma ? 1 : 0, p, rank,
                                          (int)bases.size(), stage_elems, S(st));
  });
  m.def("ar_alloc", [](int64_t bytes) {
    void* p = nullptr;
    const int rc = drtc::ar_alloc(&p, bytes);
    if (rc) throw std::runtime_error("ar_alloc failed: " + std::to_string(rc));
    return (u64)p;
  });
  m.def("ar_free", [](u64 p) { return drtc::ar_free(P<void>(p)); });
  m.def("ar_ipc_get", [](u64 p) {
    char h[64];
    const int rc = drtc::ar_ipc_get(P<void>(p), h);
    if (rc) throw std::runtime_error("hipIpcGetMemHandle failed: " + std::to_string(rc));
    return py::bytes(h, 64);
  });
  m.def("ar_ipc_open", [](py::bytes handle) {
    std::string h = handle;
    if (h.size() != 64) throw std::runtime_error("bad IPC handle size");
    void* p = nullptr;
    const int rc = drtc::ar_ipc_open(h.data(), &p);
    if (rc) throw std::runtime_error("hipIpcOpenMemHandle failed: " + std::to_string(rc));
    return (u64)p;
  });
  m.def("ar_ipc_close", [](u64 p) { return drtc::ar_ipc_close(P<void>(p)); });
  m.def("ar_error", [](u64 base) { return drtc::ar_error(P<void>(base)); });
  m.def("midm_gemm", [](u64 y, u64 x, u64 w, u64 res, int M, int N, int K, int ldx, int ldy,
                        int ldr, int epi, int splits, u64 slab, int64_t slab_bytes, u64 st) {
    return drtc::launch_midm_gemm(P<void>(y), P<const void>(x), P<const void>(w),
                                  P<const void>(res), M, N, K, ldx, ldy, ldr, epi, splits,
                                  P<void>(slab), slab_bytes, S(st));
  });
  m.def("midm_slab_bytes",
        [](int M, int N, int splits) { return drtc::midm_slab_bytes(M, N, splits); });
  m.def("ar_set_epoch", [](u64 base, uint64_t e) { return drtc::ar_set_epoch(P<void>(base), e); });
  m.def("lt_version", &drtc::lt_version);
  m.def("lt_gemm", [](u64 y, u64 x, u64 w, int64_t M, int64_t N, int64_t K, int64_t ldx,
                      int64_t ldy, float beta, u64 st) {
    return drtc::lt_gemm(P<void>(y), P<const void>(x), P<const void>(w), M, N, K, ldx, ldy, beta,
                         S(st));
  });
  m.def("lt_set_algo", &drtc::lt_set_algo);
  m.def("skinny_glu_gemm", [](u64 y, u64 gu, u64 w, int M, int N, int K, int ldx, int ldy, int act,
                              u64 st) {
    return drtc::launch_skinny_glu_gemm(P<void>(y), P<const void>(gu), P<const void>(w), M, N, K,
                                        ldx, ldy, act, S(st));
  });
  m.def("skinny_norm_gemm", [](u64 y, u64 h, u64 x, u64 res, u64 nw, u64 w, int M, int N, int K,
                               int ldx, int ldr, int ldh, int ldy, float eps, bool gemma, u64 st) {
    return drtc::launch_skinny_norm_gemm(P<void>(y), P<void>(h), P<const void>(x),
                                         P<const void>(res), P<const void>(nw), P<const void>(w),
                                         M, N, K, ldx, ldr, ldh, ldy, eps, gemma, S(st));
  });
  m.def("skinny_gemm", [](u64 y, u64 x, u64 w, int M, int N, int K, int ldx, int ldy,
                          int variant, u64 st) {
    return drtc::launch_skinny_gemm(P<void>(y), P<const void>(x), P<const void>(w), M, N, K, ldx,
                                    ldy, variant, S(st));
  });
  m.def("lt_tune", [](u64 y, u64 x, u64 w, int64_t M, int64_t N, int64_t K, int64_t ldx,
                      int64_t ldy, int iters, int max_candidates, u64 st) {
    py::gil_scoped_release nogil;
    return drtc::lt_tune(P<void>(y), P<const void>(x), P<const void>(w), M, N, K, ldx, ldy,
                         iters, max_candidates, S(st));
  });
  m.def("sample", [](u64 out_tokens, u64 logits, int B, int V, int ld,
                     u64 temperature, u64 top_k, u64 top_p, uint64_t seed,
                     u64 step, u64 st) {
    return drtc::launch_sample(P<int>(out_tokens), P<const void>(logits), B, V, ld,
                               P<const float>(temperature), P<const int>(top_k),
                               P<const float>(top_p), seed,
                               P<const int64_t>(step), S(st));
  });
}
