// amp_torch_ops.cpp — the C ABI of include/amp_sparc.h registered as PyTorch-ROCm custom ops
// (TORCH_LIBRARY(amp)): torch.ops.amp.vamp_run / bamp_run / scamp_run /
// block_denoise / map_decide_count.  Every op checks shapes, dtypes and devices (TORCH_CHECK),
// allocates its outputs and workspace from torch's caching allocator and launches on the
// tensors' device's current HIP stream — the same entry points the ctypes host package calls,
// so both paths run the same gfx950 kernels.  Built into lib/libamp_torch_ops.so (linked
// against lib/libampsparc.so); loaded by amp_native.torch_ops().
//
// Constellation arguments: `symbols` complex128 [K] (Config.symbols, config.py:117) and `gray`
// int[K] (Config.gray), K in {1, 2, 4, 8, 16, 64}.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cmath>
#include <tuple>
#include <vector>

#include "../../include/amp_sparc.h"

namespace {

using at::Tensor;

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc == AMP_OK, what, " failed (", rc, "): ", amp_last_error());
}

// PyTorch-ROCm exposes HIP devices and streams as 'cuda' ones (the masquerading guard / stream)
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

void* stream_of(const Tensor& t) {
    return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void require_dev(const Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda(), name, ": expected a ROCm device tensor (there is no CPU path), got ", t.device());
}

// [B, len] complex64 view of a [B, len] or [B, len, 1] tensor (contiguous, conj/neg resolved)
Tensor rows_c64(const Tensor& t, int64_t B, const char* name) {
    require_dev(t, name);
    TORCH_CHECK(t.scalar_type() == at::kComplexFloat, name, ": expected complex64, got ", t.scalar_type());
    TORCH_CHECK(t.dim() == 2 || (t.dim() == 3 && t.size(2) == 1), name, ": expected [B, len] or [B, len, 1], got ",
                t.sizes());
    TORCH_CHECK(t.size(0) == B, name, ": batch ", t.size(0), " != ", B);
    return t.reshape({B, t.size(1)}).resolve_conj().resolve_neg().contiguous();
}

amp_constellation make_const(const Tensor& symbols, c10::IntArrayRef gray) {
    TORCH_CHECK(symbols.dim() == 1, "symbols: expected a 1-D tensor");
    const int64_t K = symbols.numel();
    TORCH_CHECK(K >= 1 && K <= AMP_MAX_K && (K & (K - 1)) == 0 && K != 32,
                "symbols: constellation size must be 1, 2, 4, 8, 16 or 64, got ", K);
    TORCH_CHECK((int64_t)gray.size() == K, "gray: expected ", K, " labels, got ", gray.size());
    const Tensor s = symbols.to(at::kCPU).to(at::kComplexDouble).contiguous();
    const c10::complex<double>* p = s.data_ptr<c10::complex<double>>();
    amp_constellation c{};
    c.K = (int32_t)K;
    c.symbol_bits = (int32_t)std::lround(std::log2((double)K));
    for (int64_t k = 0; k < K; ++k) {
        c.re[k] = (float)p[k].real();
        c.im[k] = (float)p[k].imag();
        c.re64[k] = p[k].real();
        c.im64[k] = p[k].imag();
        c.gray[k] = (int32_t)gray[k];
    }
    return c;
}

// sparc-mode dimensions (config.py:49-71, 132-144), n = Nr * Lout.  VAMP / BAMP / the decision
// read only n (the observation length), so they pass Nr = n, Lout = 1.
amp_dims make_dims(int64_t B, int64_t Nt, int64_t Na, int64_t Nr, int64_t Lin, int64_t Lout) {
    TORCH_CHECK(B > 0 && Nt > 0 && Na > 0 && Nr > 0 && Lin > 0 && Lout > 0, "bad dimensions");
    TORCH_CHECK(Nt % Na == 0, "Na must divide Nt (config.py:133)");
    amp_dims d{};
    d.B = (int32_t)B; d.Nt = (int32_t)Nt; d.Na = (int32_t)Na; d.Nr = (int32_t)Nr; d.Lin = (int32_t)Lin;
    d.Lout = (int32_t)Lout;
    d.N = (int32_t)(Nt * Lin); d.n = (int32_t)(Nr * Lout); d.L = (int32_t)(Na * Lin); d.M = (int32_t)(Nt / Na);
    return d;
}

Tensor workspace(size_t bytes, const Tensor& like) {
    return at::empty({(int64_t)std::max<size_t>(bytes, 256)}, like.options().dtype(at::kByte));
}

// status record (amp_status) as int32 [4]: T, nan_state, stopped, gemm (AMP_ARITH_*)
Tensor status_tensor(const Tensor& like) { return at::zeros({8}, like.options().dtype(at::kInt)); }

// ---- amp::vamp_run — VAMP.forward (vamp.py:159-187) without the decision -------------------
std::tuple<Tensor, Tensor, Tensor, Tensor> vamp_run(const Tensor& U, const Tensor& s, const Tensor& Vh,
                                                    const Tensor& y, double noise_var, double sparsity, int64_t Nt,
                                                    int64_t Na, int64_t max_iter, const Tensor& symbols,
                                                    c10::IntArrayRef gray, int64_t engine) {
    require_dev(U, "U");
    require_dev(s, "s");
    require_dev(Vh, "Vh");
    const DevGuard guard(y.device());
    TORCH_CHECK(U.dim() == 2 && Vh.dim() == 2, "U [n, k] and Vh [k, N] must be 2-D");
    TORCH_CHECK(U.scalar_type() == at::kComplexFloat && Vh.scalar_type() == at::kComplexFloat, "U, Vh: complex64");
    TORCH_CHECK(s.scalar_type() == at::kFloat, "s: float32");
    const int64_t n = U.size(0), k = U.size(1), N = Vh.size(1);
    TORCH_CHECK(Vh.size(0) == k && s.numel() == k, "U [n, k], s [k], Vh [k, N] disagree: ", U.sizes(), s.sizes(),
                Vh.sizes());
    TORCH_CHECK(N % Nt == 0, "N = ", N, " is not a multiple of Nt = ", Nt);
    const int64_t B = y.size(0), Lin = N / Nt;
    TORCH_CHECK(max_iter > 0, "max_iter must be positive");
    const Tensor yy = rows_c64(y, B, "y");
    TORCH_CHECK(yy.size(1) == n, "y: length ", yy.size(1), " != n = ", n);
    amp_dims d = make_dims(B, Nt, Na, n, Lin, 1);
    const amp_constellation c = make_const(symbols, gray);
    const Tensor Uc = U.resolve_conj().resolve_neg().contiguous(), Vc = Vh.resolve_conj().resolve_neg().contiguous();
    const Tensor sc = s.reshape({k}).contiguous();
    Tensor r = at::empty({B, N}, yy.options()), xm = at::empty({B, N}, yy.options());
    Tensor var = at::empty({B, N}, yy.options().dtype(at::kFloat));
    Tensor st = status_tensor(yy);
    const size_t wsb = amp_vamp_workspace_bytes(&d, (int32_t)k, (int32_t)max_iter);
    TORCH_CHECK(wsb > 0, "amp_vamp_workspace_bytes: invalid dimensions");
    Tensor ws = workspace(wsb, yy);
    amp_vamp_args a{};
    a.U = Uc.data_ptr(); a.s = sc.data_ptr(); a.Vh = Vc.data_ptr(); a.y = yy.data_ptr();
    a.k = (int32_t)k; a.max_iter = (int32_t)max_iter; a.engine = (int32_t)engine;
    a.noise_var = noise_var; a.sparsity = sparsity;
    a.r = r.data_ptr(); a.xmmse = xm.data_ptr(); a.var = var.data_ptr(); a.status = st.data_ptr();
    a.ws = ws.data_ptr(); a.ws_bytes = (size_t)ws.numel();
    check_rc(amp_vamp_run(&d, &c, &a, stream_of(yy)), "amp_vamp_run");
    return {r, xm, var, st.slice(0, 0, 4)};
}

// ---- amp::bamp_run — BAMP.forward (bamp.py:116-143) without the decision ------------------
std::tuple<Tensor, Tensor, Tensor, Tensor> bamp_run(const Tensor& H, const Tensor& y, double noise_var, int64_t Nt,
                                                    int64_t Na, int64_t max_iter, const Tensor& symbols,
                                                    c10::IntArrayRef gray, int64_t denoiser, double P0, double Ps) {
    require_dev(H, "H");
    const DevGuard guard(y.device());
    TORCH_CHECK(H.dim() == 2 && H.scalar_type() == at::kComplexFloat, "H: complex64 [n, N]");
    const int64_t n = H.size(0), N = H.size(1), B = y.size(0);
    TORCH_CHECK(N % Nt == 0, "N = ", N, " is not a multiple of Nt = ", Nt);
    const int64_t Lin = N / Nt;
    const Tensor yy = rows_c64(y, B, "y");
    TORCH_CHECK(yy.size(1) == n, "y: length ", yy.size(1), " != n = ", n);
    TORCH_CHECK(max_iter > 0 && (denoiser == 0 || denoiser == 1), "max_iter > 0, denoiser 0 or 1");
    amp_dims d = make_dims(B, Nt, Na, n, Lin, 1);
    const amp_constellation c = make_const(symbols, gray);
    const Tensor Hc = H.resolve_conj().resolve_neg().contiguous();
    Tensor xmap = at::empty({B, N}, yy.options()), xm = at::empty({B, N}, yy.options());
    Tensor var = at::empty({B, N}, yy.options().dtype(at::kFloat));
    Tensor st = status_tensor(yy);
    Tensor ws = workspace(amp_bamp_workspace_bytes(&d, (int32_t)max_iter), yy);
    amp_bamp_args a{};
    a.H = Hc.data_ptr(); a.y = yy.data_ptr(); a.max_iter = (int32_t)max_iter; a.denoiser = (int32_t)denoiser;
    a.noise_var = noise_var; a.xmap = xmap.data_ptr(); a.xmmse = xm.data_ptr(); a.var = var.data_ptr();
    a.status = st.data_ptr(); a.ws = ws.data_ptr(); a.ws_bytes = (size_t)ws.numel();
    a.P0 = (float)P0; a.Ps = (float)Ps;
    check_rc(amp_bamp_run(&d, &c, &a, stream_of(yy)), "amp_bamp_run");
    return {xmap, xm, var, st.slice(0, 0, 4)};
}

// ---- amp::scamp_run — SCAMP.forward (scamp.py:77-107) without the decision ----------------
std::tuple<Tensor, Tensor, Tensor, Tensor> scamp_run(const Tensor& W, const Tensor& A, const Tensor& y,
                                                     double noise_var, int64_t Nt, int64_t Na, int64_t max_iter,
                                                     const Tensor& symbols, c10::IntArrayRef gray) {
    require_dev(W, "W");
    require_dev(A, "A");
    const DevGuard guard(y.device());
    TORCH_CHECK(W.dim() == 2 && W.scalar_type() == at::kFloat, "W: float32 [Lout, Lin]");
    TORCH_CHECK(A.dim() == 2 && A.scalar_type() == at::kComplexFloat, "A: complex64 [n, N]");
    const int64_t Lout = W.size(0), Lin = W.size(1), n = A.size(0), N = A.size(1), B = y.size(0);
    TORCH_CHECK(N == Nt * Lin, "A: N = ", N, " != Nt * Lin = ", Nt * Lin);
    TORCH_CHECK(n % Lout == 0, "A: n = ", n, " is not a multiple of Lout = ", Lout);
    const Tensor yy = rows_c64(y, B, "y");
    TORCH_CHECK(yy.size(1) == n, "y: length ", yy.size(1), " != n = ", n);
    TORCH_CHECK(max_iter > 0, "max_iter must be positive");
    amp_dims d = make_dims(B, Nt, Na, n / Lout, Lin, Lout);
    const amp_constellation c = make_const(symbols, gray);
    const Tensor Wc = W.contiguous(), Ac = A.resolve_conj().resolve_neg().contiguous();
    Tensor xmap = at::empty({B, N}, yy.options()), xm = at::empty({B, N}, yy.options());
    Tensor psi = at::empty({B, Lin}, yy.options().dtype(at::kFloat));
    Tensor st = status_tensor(yy);
    Tensor ws = workspace(amp_scamp_workspace_bytes(&d, (int32_t)max_iter), yy);
    amp_scamp_args a{};
    a.W = Wc.data_ptr(); a.A = Ac.data_ptr(); a.y = yy.data_ptr(); a.max_iter = (int32_t)max_iter;
    a.noise_var = noise_var; a.xmap = xmap.data_ptr(); a.xmmse = xm.data_ptr(); a.psi = psi.data_ptr();
    a.status = st.data_ptr(); a.ws = ws.data_ptr(); a.ws_bytes = (size_t)ws.numel();
    check_rc(amp_scamp_run(&d, &c, &a, stream_of(yy)), "amp_scamp_run");
    return {xmap, xm, psi, st.slice(0, 0, 4)};
}

// ---- amp::block_denoise — segmented_denoiser (vamp.py:96-119, bamp.py:66-77, scamp.py:61-68)
// mode 0: tau a 0-dim / 1-element tensor (VAMP sigma2); 1: per-element cov (BAMP, tau = cov/2);
// 2: per-element tau_use, mean only (SCAMP; the var output is empty).
std::tuple<Tensor, Tensor> block_denoise(const Tensor& r, const Tensor& tau, int64_t mode, int64_t Nt, int64_t Na,
                                         const Tensor& symbols, c10::IntArrayRef gray) {
    TORCH_CHECK(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
    const DevGuard guard(r.device());
    const int64_t B = r.size(0);
    const Tensor rr = rows_c64(r, B, "r");
    const int64_t N = rr.size(1);
    TORCH_CHECK(N % Nt == 0, "r: length ", N, " is not a multiple of Nt = ", Nt);
    amp_dims d = make_dims(B, Nt, Na, 1, N / Nt, 1);
    const amp_constellation c = make_const(symbols, gray);
    float ts = 0.f;
    Tensor tv;
    if (mode == 0) {
        TORCH_CHECK(tau.numel() == 1, "mode 0: tau must hold one value");
        ts = tau.to(at::kFloat).item<float>();
    } else {
        require_dev(tau, "tau");
        TORCH_CHECK(tau.numel() == B * N, "tau: expected ", B * N, " values, got ", tau.numel());
        tv = tau.reshape({B, N}).to(at::kFloat).contiguous();
    }
    Tensor xm = at::empty({B, N}, rr.options());
    Tensor var = mode == 2 ? at::empty({0}, rr.options().dtype(at::kFloat))
                           : at::empty({B, N}, rr.options().dtype(at::kFloat));
    Tensor ws = workspace(amp_block_denoise_workspace_bytes(&d), rr);
    check_rc(amp_block_denoise(&d, &c, rr.data_ptr(), (int32_t)mode, ts, mode == 0 ? nullptr : tv.data_ptr(),
                               xm.data_ptr(), mode == 2 ? nullptr : var.data_ptr(), ws.data_ptr(),
                               (size_t)ws.numel(), stream_of(rr)),
             "amp_block_denoise");
    return {xm, var};
}

// ---- amp::map_decide_count — Loss.error_rate (loss.py:67-179) for generator_mode='sparc' ----
// Returns amp_counts as float64 [13] (ier, ser, iber, sber, ver, verf, verm, verL, fer, mse,
// msef, msem, mseL), the integer counters exact.
Tensor map_decide_count(const Tensor& xmap, const Tensor& xmmse, const Tensor& x, const Tensor& sym,
                        const Tensor& idx, int64_t Nt, int64_t Na, const Tensor& symbols, c10::IntArrayRef gray) {
    const DevGuard guard(xmap.device());
    const int64_t B = xmap.size(0);
    const Tensor a = rows_c64(xmap, B, "xmap"), b = rows_c64(xmmse, B, "xmmse"), t = rows_c64(x, B, "x");
    const int64_t N = a.size(1);
    TORCH_CHECK(b.size(1) == N && t.size(1) == N, "xmap, xmmse, x must have the same length");
    TORCH_CHECK(N % Nt == 0, "length ", N, " is not a multiple of Nt = ", Nt);
    const int64_t Lin = N / Nt;
    amp_dims d = make_dims(B, Nt, Na, 1, Lin, 1);
    const amp_constellation c = make_const(symbols, gray);
    require_dev(sym, "sym");
    require_dev(idx, "idx");
    TORCH_CHECK(sym.scalar_type() == at::kLong && idx.scalar_type() == at::kLong, "sym, idx: int64");
    TORCH_CHECK(sym.numel() == B * d.L && idx.numel() == B * d.L, "sym / idx: expected ", B * d.L, " labels");
    const Tensor sy = sym.contiguous(), ix = idx.contiguous();
    const int32_t ibits = (int32_t)std::ceil(std::log2((double)(Lin * B * Na)));   // loss.py:20
    Tensor counts = at::zeros({13}, a.options().dtype(at::kDouble));
    static_assert(sizeof(amp_counts) == 13 * 8, "amp_counts layout");
    Tensor ws = workspace(amp_map_decide_workspace_bytes(&d), a);
    check_rc(amp_map_decide_count(&d, &c, a.data_ptr(), b.data_ptr(), t.data_ptr(), sy.data_ptr(), ix.data_ptr(), ibits,
                                  counts.data_ptr(), nullptr, ws.data_ptr(), (size_t)ws.numel(), stream_of(a)),
             "amp_map_decide_count");
    // the first 9 fields are int64: reinterpret them and convert, on the device
    Tensor raw = counts.slice(0, 0, 13);
    Tensor ints = raw.slice(0, 0, 9).view(at::kLong).to(at::kDouble);
    return at::cat({ints, raw.slice(0, 9, 13)});
}

}  // namespace

TORCH_LIBRARY(amp, m) {
    m.def("vamp_run(Tensor U, Tensor s, Tensor Vh, Tensor y, float noise_var, float sparsity, int Nt, int Na, "
          "int max_iter, Tensor symbols, int[] gray, int engine=0) -> (Tensor r, Tensor xmmse, Tensor var, "
          "Tensor status)");
    m.def("bamp_run(Tensor H, Tensor y, float noise_var, int Nt, int Na, int max_iter, Tensor symbols, int[] gray, "
          "int denoiser=0, float P0=0.0, float Ps=0.0) -> (Tensor xmap, Tensor xmmse, Tensor var, Tensor status)");
    m.def("scamp_run(Tensor W, Tensor A, Tensor y, float noise_var, int Nt, int Na, int max_iter, Tensor symbols, "
          "int[] gray) -> (Tensor xmap, Tensor xmmse, Tensor psi, Tensor status)");
    m.def("block_denoise(Tensor r, Tensor tau, int mode, int Nt, int Na, Tensor symbols, int[] gray) -> "
          "(Tensor xmmse, Tensor var)");
    m.def("map_decide_count(Tensor xmap, Tensor xmmse, Tensor x, Tensor sym, Tensor idx, int Nt, int Na, "
          "Tensor symbols, int[] gray) -> Tensor");
}

TORCH_LIBRARY_IMPL(amp, CUDA, m) {
    m.impl("vamp_run", &vamp_run);
    m.impl("bamp_run", &bamp_run);
    m.impl("scamp_run", &scamp_run);
    m.impl("block_denoise", &block_denoise);
    m.impl("map_decide_count", &map_decide_count);
}
