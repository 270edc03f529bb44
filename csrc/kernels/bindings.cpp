// pybind11 launcher table for the HIP kernels (module llm_consensus_amd._lib._llmc_hip).
//
// Every entry takes raw device pointers (uintptr_t from torch.Tensor.data_ptr()) and the HIP
// stream handle (torch.cuda.current_stream().cuda_stream), launches asynchronously and raises
// on a launch error. No torch headers: the module builds in seconds and is graph-capturable
// (launches land on whatever stream torch is capturing).
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>

#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
typedef uintptr_t ptr;

extern "C" {
int llmc_rmsnorm(const void*, const void*, void*, int, int, int, int, float, hipStream_t);
int llmc_embedding(const void*, const void*, void*, int, int, int, hipStream_t);
int llmc_lane_exchange_check(const void*, void*, int, hipStream_t);
int llmc_silu_mul_interleaved(const void*, void*, int, int, hipStream_t);
int llmc_gemv(int, const void*, int, const void*, float, const void*, void*, int, int, int, int, int, hipStream_t);
int llmc_gemvm(int, const void*, int, const void*, float, const void*, void*, int, int, int, int, int, hipStream_t);
int llmc_moe_gemvm(int, const void*, int, const void*, float, const void*, const void*, int, int, void*, int, int, int,
                   int, hipStream_t);
int llmc_gemm(const void*, int, const void*, int, void*, int, int, int, int, int, hipStream_t);
int llmc_gemm_t128(const void*, int, const void*, int, void*, int, int, int, int, int, hipStream_t);
int llmc_gemm_narrow(const void*, int, const void*, int, void*, int, int, int, int, int, hipStream_t);
int llmc_gemm_kind(const void*, int, const void*, int, void*, int, int, int, int, int, int, hipStream_t);
int llmc_gemm_plan(int, int);
int llmc_rope_kv_write(const void*, int, void*, int, const void*, const void*, const void*, void*, void*, const void*,
                       int, int, int, int, int, hipStream_t);
int llmc_attn_decode_groups(int);
int llmc_qkv_attn_check(int, int, int, int);
int llmc_qkv_attn(const void*, const void*, float, const void*, int, void*, void*, void*, const void*, const void*,
                  const void*, const void*, const void*, int, const void*, void*, void*, void*, int, int, int, int, int,
                  int, int, int, float, void*, void*, void*, int, const void*, void*, int, const void* const*, void*,
                  int, int, size_t, hipStream_t);
int llmc_attn_oproj_check(int, int, int, int, int, int);
int llmc_attn_oproj_form(int, int, int, int, int, int, int, int);
int llmc_attn_oproj(const void*, const void*, const void*, const void*, int, const void*, const void*, void*, void*,
                    void*, void*, void*, void*, void*, int, int, int, int, int, int, int, int, float, int, void*,
                    int, const void* const*, void*, int, int, size_t, const void*, const void*, float, int, int,
                    void*, void*, void*, void*, hipStream_t);
int llmc_attn_decode(const void*, int, const void*, const void*, const void*, int, const void*, void*, void*, void*,
                     int, int, int, int, int, int, int, int, int, int, float, int, void*, hipStream_t);
int llmc_gemv_qkv_rope(int, const void*, int, const void*, float, const void*, int, int, void*, int, void*, void*,
                       const void*, const void*, const void*, const void*, int, int, int, int, int, hipStream_t);
int llmc_attn_prefill(const void*, int, const void*, const void*, const void*, int, const void*, const void*,
                      const void*, void*, int, int, int, int, int, int, int, float, int, int, void*, void*, int,
                      int, hipStream_t);
int llmc_attn_prefill_form(int, int, int, int, int, int, int);
int llmc_attn_prefill_plan(int, int, int, int, int, int, int, int*);
int64_t llmc_attn_prefill_counters(int, int, int, int);
int llmc_sample(const void*, int64_t, int, int, const void*, const void*, const void*, const void*, const void*, void*,
                void*, void*, void*, void*, void*, const void*, int, int, void*, void*, int, int, hipStream_t);
int llmc_sample_parts();
int llmc_moe_route(const void*, int, int, int, void*, void*, hipStream_t);
int llmc_moe_down_combine(int, const void*, int, const void*, const void*, const void*, void*, int, int, int, int,
                          hipStream_t);
int llmc_moe_router(const void*, int, const void*, float, const void*, int, int, int, int, void*, void*, hipStream_t);
int llmc_moe_align(const void*, int, int, int, int, void*, void*, void*, void*, hipStream_t);
int llmc_moe_gemm(const void*, int, int, const void*, const void*, const void*, const void*, void*, int, int, int, int,
                  int, int, int, hipStream_t);
int llmc_moe_combine(const void*, const void*, const void*, void*, int, int, int, hipStream_t);
int llmc_moe_gemv(int, const void*, int, const void*, float, const void*, const void*, int, void*, int, int, int, int,
                  hipStream_t);
int llmc_moe_ep_localize(const void*, const void*, int, int, int, void*, void*, hipStream_t);
int llmc_moe_ep_dispatch(const void*, int, int, int, int, void*, void*, void*, void*, hipStream_t);
int llmc_gather_rows(const void*, int, const void*, int, int, int, void*, int, hipStream_t);
int llmc_moe_route_fused(const void*, int, const void*, int, int, int, int, void*, void*, hipStream_t);
int llmc_gemv_sweep(int, const void*, const void*, const void*, void*, int, int, hipStream_t);
size_t llmc_car_sig_bytes();
int llmc_car_alloc(size_t, void**);
int llmc_car_free(void*);
int llmc_ipc_handle(void*, void*);
int llmc_ipc_handle_size();
int llmc_ipc_open(const void*, void**);
int llmc_ipc_close(void*);
int llmc_car_timed_out(void*, int*);
int llmc_car_max_wait(void*, uint32_t*);
int llmc_car_host_alloc(void**, void**);
int llmc_car_host_free(void*);
int llmc_car_host_get(const void*, int);
void llmc_car_host_set(void*, int, int);
int llmc_car_host_word(int);
size_t llmc_car_timeout_off();
int llmc_car_reset(void*, size_t);
size_t llmc_car_oneshot_max(size_t);
int llmc_gemv_ar(int, const void*, int, const void*, void*, int, int, int, const void* const*, void*, int, int, size_t,
                 hipStream_t);
int llmc_stream_cu_mask(int, const uint32_t*, int, void**);
int llmc_can_access_peer(int, int, int*);
int llmc_car_twoshot(const void* const*, void*, int, int, size_t, int, const void*, void*, long, int, int, hipStream_t);
int llmc_car_allreduce(const void* const*, void*, int, int, size_t, void*, size_t, hipStream_t);
int llmc_car_allgather(const void* const*, void*, int, int, size_t, const void*, void*, size_t, hipStream_t);
}

static inline void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string("llmc HIP launch failed: ") + what + " rc=" + std::to_string(rc);
    if (rc > 0) msg += std::string(" (") + hipGetErrorString(static_cast<hipError_t>(rc)) + ")";
    throw std::runtime_error(msg);
  }
}
#define P(x) reinterpret_cast<void*>(x)
#define S(x) reinterpret_cast<hipStream_t>(x)

PYBIND11_MODULE(_llmc_hip, m) {
  m.doc() = "llm_consensus_amd gfx950 HIP kernels (raw-pointer launchers)";
  m.def("rmsnorm", [](ptr x, ptr w, ptr y, int T, int H, int xs, int ys, float eps, ptr s) {
    check(llmc_rmsnorm(P(x), P(w), P(y), T, H, xs, ys, eps, S(s)), "rmsnorm");
  });
  m.def("lane_exchange_check", [](ptr in, ptr out, int nb, ptr s) {
    check(llmc_lane_exchange_check(P(in), P(out), nb, S(s)), "lane_exchange_check");
  });
  m.def("embedding", [](ptr ids, ptr table, ptr out, int T, int H, int V, ptr s) {
    check(llmc_embedding(P(ids), P(table), P(out), T, H, V, S(s)), "embedding");
  });
  m.def("silu_mul_interleaved", [](ptr gu, ptr y, int T, int I, ptr s) {
    check(llmc_silu_mul_interleaved(P(gu), P(y), T, I, S(s)), "silu_mul");
  });
  m.def("gemv", [](int M, ptr x, int xs, ptr nw, float eps, ptr W, ptr out, int os, int N, int K, int epi, int mfma,
                   ptr s) {
    check(llmc_gemv(M, P(x), xs, P(nw), eps, P(W), P(out), os, N, K, epi, mfma, S(s)), "gemv");
  });
  m.def("moe_gemvm", [](int P, ptr x, int xs, ptr nw, float eps, ptr W, ptr ids, int x_div, int E, ptr out, int os,
                        int N, int K, int epi, ptr s) {
    check(llmc_moe_gemvm(P, P(x), xs, P(nw), eps, P(W), P(ids), x_div, E, P(out), os, N, K, epi, S(s)), "moe_gemvm");
  });
  m.def("gemvm", [](int M, ptr x, int xs, ptr nw, float eps, ptr W, ptr out, int os, int N, int K, int epi, int form,
                    ptr s) {
    check(llmc_gemvm(M, P(x), xs, P(nw), eps, P(W), P(out), os, N, K, epi, form, S(s)), "gemvm");
  });
  m.def("gemm", [](ptr A, int lda, ptr W, int ldw, ptr C, int ldc, int M, int N, int K, int epi, ptr s) {
    check(llmc_gemm(P(A), lda, P(W), ldw, P(C), ldc, M, N, K, epi, S(s)), "gemm");
  });
  m.def("gemm_t128", [](ptr A, int lda, ptr W, int ldw, ptr C, int ldc, int M, int N, int K, int epi, ptr s) {
    check(llmc_gemm_t128(P(A), lda, P(W), ldw, P(C), ldc, M, N, K, epi, S(s)), "gemm_t128");
  });
  m.def("gemm_kind", [](ptr A, int lda, ptr W, int ldw, ptr C, int ldc, int M, int N, int K, int epi, int kind, ptr s) {
    check(llmc_gemm_kind(P(A), lda, P(W), ldw, P(C), ldc, M, N, K, epi, kind, S(s)), "gemm_kind");
  });
  m.def("gemm_plan", [](int M, int N) { return llmc_gemm_plan(M, N); });
  m.def("gemm_narrow", [](ptr A, int lda, ptr W, int ldw, ptr C, int ldc, int M, int N, int K, int epi, ptr s) {
    check(llmc_gemm_narrow(P(A), lda, P(W), ldw, P(C), ldc, M, N, K, epi, S(s)), "gemm_narrow");
  });
  m.def("rope_kv_write", [](ptr qkv, int qs, ptr qo, int qos, ptr pos, ptr cos_t, ptr sin_t, ptr kc, ptr vc,
                            ptr slots, int T, int nh, int nkv, int D, int bs, ptr s) {
    check(llmc_rope_kv_write(P(qkv), qs, P(qo), qos, P(pos), P(cos_t), P(sin_t), P(kc), P(vc), P(slots), T, nh, nkv, D,
                             bs, S(s)),
          "rope_kv_write");
  });
  m.def("attn_decode_groups", [](int max_chunks) { return llmc_attn_decode_groups(max_chunks); });
  m.def("qkv_attn_check", [](int nh, int nkv, int D, int K) { return llmc_qkv_attn_check(nh, nkv, D, K); });
  m.def("qkv_attn", [](ptr x, ptr nw, float eps, ptr W, int K, ptr qo, ptr kc, ptr vc, ptr pos, ptr slots, ptr cos_t,
                       ptr sin_t, ptr bt, int bt_len, ptr sl, ptr part, ptr ctr, ptr out, int nh, int nkv, int D, int bs,
                       int nblocks, int chunk, int gc, int max_chunks, float scale, ptr fault, ptr gran, ptr hctr,
                       int o_mode, ptr w_o, ptr h, int o_n, const std::vector<ptr>& bases, ptr host, int rank, int world,
                       size_t cap, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_qkv_attn(P(x), P(nw), eps, P(W), K, P(qo), P(kc), P(vc), P(pos), P(slots), P(cos_t), P(sin_t), P(bt),
                        bt_len, P(sl), P(part), P(ctr), P(out), nh, nkv, D, bs, nblocks, chunk, gc, max_chunks, scale,
                        P(fault), P(gran), P(hctr), o_mode, P(w_o), P(h), o_n, b.empty() ? nullptr : b.data(), P(host),
                        rank, world, cap, S(s)),
          "qkv_attn");
  });
  m.def("attn_oproj_check", [](int H, int nh, int nkv, int D, int nc, int K_o) {
    return llmc_attn_oproj_check(H, nh, nkv, D, nc, K_o);
  });
  m.def("attn_oproj_form", [](int H, int nh, int nkv, int D, int nc, int chunk, int mode, int world) {
    return llmc_attn_oproj_form(H, nh, nkv, D, nc, chunk, mode, world);
  });
  m.def("attn_oproj", [](ptr q, ptr kc, ptr vc, ptr bt, int bt_len, ptr sl, ptr w_o, ptr h, ptr attn_out, ptr part,
                         ptr handoff, ptr tile_part, ptr ctr, ptr fault, int H, int nh, int nkv, int D, int bs,
                         int nblocks, int chunk, int nc, float scale, int mode, ptr stamps, int add_resid,
                         const std::vector<ptr>& bases, ptr host, int rank, int world, size_t cap, ptr rt_norm,
                         ptr rt_wr, float rt_eps, int rt_E, int rt_k, ptr rt_w, ptr rt_ids, ptr rt_part,
                         ptr rt_epoch, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_attn_oproj(P(q), P(kc), P(vc), P(bt), bt_len, P(sl), P(w_o), P(h), P(attn_out), P(part), P(handoff),
                          P(tile_part), P(ctr), P(fault), H, nh, nkv, D, bs, nblocks, chunk, nc, scale, mode, P(stamps),
                          add_resid, b.empty() ? nullptr : b.data(), P(host), rank, world, cap, P(rt_norm), P(rt_wr),
                          rt_eps, rt_E, rt_k, P(rt_w), P(rt_ids), P(rt_part), P(rt_epoch), S(s)),
          "attn_oproj");
  });
  m.def("attn_decode", [](ptr q, int qs, ptr kc, ptr vc, ptr bt, int bts, ptr sl, ptr part, ptr ctr, ptr out, int os,
                          int B, int nh, int nkv, int D, int bs, int nblocks, int chunk, int grid_chunks,
                          int max_chunks, float scale, int fused, ptr fault, ptr s) {
    check(llmc_attn_decode(P(q), qs, P(kc), P(vc), P(bt), bts, P(sl), P(part), P(ctr), P(out), os, B, nh, nkv, D, bs,
                           nblocks, chunk, grid_chunks, max_chunks, scale, fused, P(fault), S(s)),
          "attn_decode");
  });
  m.def("gemv_qkv_rope", [](int M, ptr x, int xs, ptr nw, float eps, ptr W, int N, int K, ptr qo, int qos, ptr kc,
                            ptr vc, ptr pos, ptr slots, ptr cos_t, ptr sin_t, int nh, int nkv, int D, int bs,
                            int mfma, ptr s) {
    check(llmc_gemv_qkv_rope(M, P(x), xs, P(nw), eps, P(W), N, K, P(qo), qos, P(kc), P(vc), P(pos), P(slots),
                             P(cos_t), P(sin_t), nh, nkv, D, bs, mfma, S(s)),
          "gemv_qkv_rope");
  });
  m.def("attn_prefill", [](ptr q, int qs, ptr kc, ptr vc, ptr bt, int bts, ptr qst, ptr ql, ptr cl, ptr out, int os,
                           int B, int max_qlen, int nh, int nkv, int D, int bs, float scale, int ksplit, int kmin,
                           ptr part, ptr counters, int T, int form, ptr s) {
    check(llmc_attn_prefill(P(q), qs, P(kc), P(vc), P(bt), bts, P(qst), P(ql), P(cl), P(out), os, B, max_qlen, nh, nkv,
                            D, bs, scale, ksplit, kmin, P(part), P(counters), T, form, S(s)),
          "attn_prefill");
  });
  m.def("attn_prefill_counters", [](int B, int max_qlen, int nh, int nkv) {
    return llmc_attn_prefill_counters(B, max_qlen, nh, nkv);
  });
  m.def("attn_prefill_form", [](int B, int T, int nh, int nkv, int ksplit, int D, int bs) {
    return llmc_attn_prefill_form(B, T, nh, nkv, ksplit, D, bs);
  });
  m.def("attn_prefill_plan", [](int B, int max_qlen, int max_ctx, int nh, int nkv, int D, int bs) {
    int kmin = 0;
    const int k = llmc_attn_prefill_plan(B, max_qlen, max_ctx, nh, nkv, D, bs, &kmin);
    return std::make_pair(k, kmin);
  });
  m.def("sample", [](ptr logits, int64_t rs, int B, int V, ptr it, ptr tk, ptr tp, ptr seeds, ptr pos, ptr wv, ptr wi,
                     ptr next, ptr tin, ptr sl, ptr slots, ptr bt, int bts, int bs, ptr ot, ptr oc, int cap,
                     int use_topkp, ptr s) {
    check(llmc_sample(P(logits), rs, B, V, P(it), P(tk), P(tp), P(seeds), P(pos), P(wv), P(wi), P(next), P(tin), P(sl),
                      P(slots), P(bt), bts, bs, P(ot), P(oc), cap, use_topkp, S(s)),
          "sample");
  });
  m.def("sample_parts", []() { return llmc_sample_parts(); });
  m.def("moe_route", [](ptr logits, int T, int E, int k, ptr w, ptr ids, ptr s) {
    check(llmc_moe_route(P(logits), T, E, k, P(w), P(ids), S(s)), "moe_route");
  });
  m.def("moe_down_combine", [](int T, ptr act, int as, ptr W, ptr ids, ptr w, ptr h, int hs, int N, int K, int k,
                               ptr s) {
    check(llmc_moe_down_combine(T, P(act), as, P(W), P(ids), P(w), P(h), hs, N, K, k, S(s)), "moe_down_combine");
  });
  m.def("moe_router", [](ptr x, int xs, ptr nw, float eps, ptr Wr, int T, int E, int H, int k, ptr w, ptr ids, ptr s) {
    check(llmc_moe_router(P(x), xs, P(nw), eps, P(Wr), T, E, H, k, P(w), P(ids), S(s)), "moe_router");
  });
  m.def("moe_align", [](ptr ids, int T, int k, int E, int tile, ptr sorted_rows, ptr tile_expert, ptr tile_count,
                        ptr counts, ptr s) {
    check(llmc_moe_align(P(ids), T, k, E, tile, P(sorted_rows), P(tile_expert), P(tile_count), P(counts), S(s)),
          "moe_align");
  });
  m.def("moe_gemm", [](ptr A, int lda, int a_rows, ptr W, ptr sorted_rows, ptr tile_expert, ptr tile_count, ptr C,
                       int ldc, int N, int K, int max_tiles, int a_row_div, int epi, int tile, ptr s) {
    check(llmc_moe_gemm(P(A), lda, a_rows, P(W), P(sorted_rows), P(tile_expert), P(tile_count), P(C), ldc, N, K,
                        max_tiles, a_row_div, epi, tile, S(s)),
          "moe_gemm");
  });
  m.def("moe_combine", [](ptr y, ptr w, ptr rows, ptr out, int T, int k, int H, ptr s) {
    check(llmc_moe_combine(P(y), P(w), P(rows), P(out), T, k, H, S(s)), "moe_combine");
  });
  m.def("moe_gemv", [](int npairs, ptr x, int xs, ptr nw, float eps, ptr W, ptr ids, int x_div, ptr out, int os,
                       int N, int K, int epi, ptr s) {
    check(llmc_moe_gemv(npairs, P(x), xs, P(nw), eps, P(W), P(ids), x_div, P(out), os, N, K, epi, S(s)), "moe_gemv");
  });
  m.def("moe_ep_dispatch", [](ptr ids, int npairs, int El, int n, int cap, ptr sp, ptr se, ptr slot, ptr cnt, ptr s) {
    check(llmc_moe_ep_dispatch(P(ids), npairs, El, n, cap, P(sp), P(se), P(slot), P(cnt), S(s)), "moe_ep_dispatch");
  });
  m.def("moe_route_fused", [](ptr x, int xs, ptr wr, int T, int E, int H, int k, ptr w, ptr ids, ptr s) {
    check(llmc_moe_route_fused(P(x), xs, P(wr), T, E, H, k, P(w), P(ids), S(s)), "moe_route_fused");
  });
  m.def("gather_rows", [](ptr x, int xs, ptr rows, int M, int div, int H, ptr out, int os, ptr s) {
    check(llmc_gather_rows(P(x), xs, P(rows), M, div, H, P(out), os, S(s)), "gather_rows");
  });
  m.def("moe_ep_localize", [](ptr ids, ptr w, int n, int e0, int nl, ptr lids, ptr lw, ptr s) {
    check(llmc_moe_ep_localize(P(ids), P(w), n, e0, nl, P(lids), P(lw), S(s)), "moe_ep_localize");
  });
  m.def("device_synchronize", []() { check(static_cast<int>(hipDeviceSynchronize()), "hipDeviceSynchronize"); });
  // ---- K13 custom all-reduce / all-gather over IPC peer buffers ----
  m.def("car_sig_bytes", []() { return llmc_car_sig_bytes(); });
  m.def("car_alloc", [](size_t cap) {
    void* p = nullptr;
    check(llmc_car_alloc(cap, &p), "car_alloc");
    return reinterpret_cast<ptr>(p);
  });
  m.def("car_free", [](ptr p) { check(llmc_car_free(P(p)), "car_free"); });
  m.def("ipc_handle", [](ptr p) {
    std::string h(static_cast<size_t>(llmc_ipc_handle_size()), '\0');
    check(llmc_ipc_handle(P(p), h.data()), "ipc_handle");
    return py::bytes(h);
  });
  m.def("ipc_open", [](py::bytes h) {
    std::string s = h;
    if (static_cast<int>(s.size()) != llmc_ipc_handle_size()) throw std::runtime_error("ipc_open: bad handle size");
    void* p = nullptr;
    check(llmc_ipc_open(s.data(), &p), "ipc_open");
    return reinterpret_cast<ptr>(p);
  });
  m.def("ipc_close", [](ptr p) { check(llmc_ipc_close(P(p)), "ipc_close"); });
  m.def("car_timed_out", [](ptr own) {
    int v = 0;
    check(llmc_car_timed_out(P(own), &v), "car_timed_out");
    return v;
  });
  m.def("car_timeout_off", []() { return llmc_car_timeout_off(); });
  m.def("car_max_wait", [](ptr own) {
    uint32_t v = 0;
    check(llmc_car_max_wait(P(own), &v), "car_max_wait");
    return v;
  });
  // host status page: (host address, device address)
  m.def("car_host_alloc", []() {
    void* h = nullptr;
    void* d = nullptr;
    check(llmc_car_host_alloc(&h, &d), "car_host_alloc");
    return py::make_tuple(reinterpret_cast<ptr>(h), reinterpret_cast<ptr>(d));
  });
  m.def("car_host_free", [](ptr h) { check(llmc_car_host_free(P(h)), "car_host_free"); });
  m.def("car_host_get", [](ptr h, int word) { return llmc_car_host_get(P(h), word); });
  m.def("car_host_set", [](ptr h, int word, int v) { llmc_car_host_set(P(h), word, v); });
  m.def("car_host_word", [](int which) { return llmc_car_host_word(which); });
  m.def("car_reset", [](ptr own, size_t cap) { check(llmc_car_reset(P(own), cap), "car_reset"); });
  m.def("car_oneshot_max", [](size_t cap) { return llmc_car_oneshot_max(cap); });
  m.def("gemv_ar", [](int M, ptr x, int xs, ptr W, ptr h, int hs, int N, int K, const std::vector<ptr>& bases,
                      ptr host, int rank, int world, size_t cap, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_gemv_ar(M, P(x), xs, P(W), P(h), hs, N, K, b.data(), P(host), rank, world, cap, S(s)), "gemv_ar");
  });
  // a stream restricted to a set of CUs (rehearsals: ranks sharing one GPU on disjoint CUs)
  m.def("stream_cu_mask", [](int device, const std::vector<uint32_t>& mask) {
    void* st = nullptr;
    check(llmc_stream_cu_mask(device, mask.data(), static_cast<int>(mask.size()), &st), "stream_cu_mask");
    return reinterpret_cast<ptr>(st);
  });
  m.def("can_access_peer", [](int dev, int peer) {
    int v = 0;
    check(llmc_can_access_peer(dev, peer, &v), "can_access_peer");
    return v;
  });
  m.def("car_twoshot", [](const std::vector<ptr>& bases, ptr host, int rank, int world, size_t cap, int mode, ptr in,
                          ptr out, long seg_stride, int seg16, int nv, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_car_twoshot(b.data(), P(host), rank, world, cap, mode, P(in), P(out), seg_stride, seg16, nv, S(s)),
          "car_twoshot");
  });
  m.def("car_allreduce", [](const std::vector<ptr>& bases, ptr host, int rank, int world, size_t cap, ptr x,
                            size_t nbytes, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_car_allreduce(b.data(), P(host), rank, world, cap, P(x), nbytes, S(s)), "car_allreduce");
  });
  m.def("car_allgather", [](const std::vector<ptr>& bases, ptr host, int rank, int world, size_t cap, ptr x, ptr out,
                            size_t nbytes, ptr s) {
    std::vector<const void*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = P(bases[i]);
    check(llmc_car_allgather(b.data(), P(host), rank, world, cap, P(x), P(out), nbytes, S(s)), "car_allgather");
  });
  m.def("gemv_sweep", [](int v, ptr x, ptr nw, ptr W, ptr out, int N, int K, ptr s) {
    check(llmc_gemv_sweep(v, P(x), P(nw), P(W), P(out), N, K, S(s)), "gemv_sweep");
  });
}
