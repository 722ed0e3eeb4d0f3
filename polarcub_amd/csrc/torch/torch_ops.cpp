// torch_ops.cpp -- the PyTorch-ROCm operator form of the drop-in boundary (the
// extension exports listed at SURVEY.md:443).  A thin host-only layer over the C ABI of
// include/polarcub_sc.h: it checks shapes, allocates outputs on the tensors' device, and launches
// on torch's current HIP stream.  No compute happens here; every op is the same device path the
// ctypes facade (polarcub_amd/sc.py) drives, so its outputs are identical to the facade's.
//
//   polarcub::sc_decode_bin_f64(xy [B,N,2] f64, frozen_mask [N] u8, frozen_val [N] u8)
//       -> (info [B,K] u8, xhat [B,N] u8)
//       BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99) for a uniform prior;
//       frozen_val[i] is the reference's frozen decision at position i (:258-262).
//   polarcub::sc_decode_qary_f64(q, xy [B,N,q] f64, frozen_mask [N] u8)
//       -> (info [B,K] u8, xhat [B,N] u8)
//       QaryPolarEncoderDecoder.decode (QaryPolarEncoderDecoder.py:90-116), frozen symbols 0.
//   polarcub::sc_decode_bin_f64.leaf(xy, frozen_mask, frozen_val)
//       -> (info [B,K] u8, xhat [B,N] u8, leaf_m [B,N,2] f64)
//       the same decode with every leaf's marginal (the reference's marginalizedUProbs capture,
//       :268-273; calcMarginalizedProbabilities, BinaryMemorylessVectorDistribution.py:52-69)
//       through pcub_sc_leaf_bin + pcub_leaf_marginals.
//   polarcub::sc_decode_bin_words(xy, frozen_words [ceil(N/32)] i32, frozen_val_words, int K)
//       -> (info [B,K] u8, xhat [B,N] u8)
//       sc_decode_bin_f64 with the masks already packed on the device and K given: no host
//       synchronisation, so it can be captured in a HIP graph; a Meta kernel gives its shapes.
//   polarcub::polar_encode_bin(u [B,N] u8) -> x [B,N] u8
//       the polar transform of every decision vector u (BinaryPolarEncoderDecoder.py:319-323,
//       polarTransformOfBits :494-516).
//   polarcub::mc_run(log2N, channel, param, frozen_mask, frozen_val, seed, cw_offset, count,
//                    chunk) -> counters [4] i64 on the masks' device
//       encodeDecodeSimulation (BinaryPolarEncoderDecoder.py:328-387) as the device pipeline
//       pcub_mc_run_bin over global codewords [cw_offset, cw_offset + count): {codewords, frame
//       errors, bit errors, 0}; channel 0 = BI-AWGN (param = sigma^2), 1 = BSC (param = p).
//
// The byte masks may live on the host or the device; K is counted on the host (the output shape
// depends on it), so a device mask costs one small copy and a synchronisation (the _words form
// avoids both).  Errors surface as c10::Error (RuntimeError in Python) naming the C entry point,
// as the ctypes facade's _lib.check does.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <tuple>

#include "polarcub_sc.h"

namespace {

void* stream_of(const at::Tensor& t) {
    return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int log2_exact(int64_t N) {
    TORCH_CHECK(N >= 2 && (N & (N - 1)) == 0, "polarcub: code length must be a power of two >= 2, got ", N);
    int n = 0;
    while ((int64_t(1) << n) < N) ++n;
    return n;
}

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc == 0, "polarcub: ", what, " failed (", rc == PCUB_EINVAL ? "invalid argument" : "HIP error",
                ", code ", rc, ")");
}

// [N] 0/1 -> ceil(N/32) u32 words on `dev` (bit i of word i/32), and the number of set bits.
std::pair<at::Tensor, int64_t> mask_words(const at::Tensor& m, int64_t N, const at::Device& dev) {
    TORCH_CHECK(m.numel() == N, "polarcub: frozen mask has ", m.numel(), " entries, expected N=", N);
    auto h = m.reshape({-1}).to(at::kCPU).ne(0).to(at::kByte).contiguous();
    const int64_t W = std::max<int64_t>(1, (N + 31) / 32);
    auto w = at::zeros({W}, at::kInt);
    const uint8_t* p = h.data_ptr<uint8_t>();
    auto* o = reinterpret_cast<uint32_t*>(w.data_ptr<int32_t>());
    int64_t ones = 0;
    for (int64_t i = 0; i < N; ++i)
        if (p[i]) {
            o[i >> 5] |= 1u << (i & 31);
            ++ones;
        }
    return {w.to(dev), ones};
}

at::Tensor unpack_words(const at::Tensor& words, int64_t B, int64_t nbits, void* s) {
    auto out = at::empty({B, nbits}, words.options().dtype(at::kByte));
    if (B > 0 && nbits > 0)
        check_rc(pcub_unpack_bits(reinterpret_cast<const uint32_t*>(words.data_ptr<int32_t>()), B, (int32_t)nbits,
                                  out.data_ptr<uint8_t>(), s),
                 "pcub_unpack_bits");
    return out;
}

void check_xy_bin(const at::Tensor& xy_in) {
    TORCH_CHECK(xy_in.is_cuda() && xy_in.scalar_type() == at::kDouble && xy_in.dim() == 3 && xy_in.size(2) == 2,
                "polarcub: xy must be a float64 [B, N, 2] device tensor");
}

// the tiled decode (the facade's and the bench's kernels) on packed device masks
std::tuple<at::Tensor, at::Tensor> decode_bin_core(const at::Tensor& xy_in, const at::Tensor& fm_words,
                                                   const at::Tensor& fv_words, int64_t K) {
    const int64_t B = xy_in.size(0), N = xy_in.size(1);
    const int n = log2_exact(N);
    auto u8 = xy_in.options().dtype(at::kByte);
    if (B == 0) return {at::empty({0, K}, u8), at::empty({0, N}, u8)};
    void* s = stream_of(xy_in);
    auto xy = xy_in.contiguous();
    const int T = pcub_sc_bin_tile(n);
    TORCH_CHECK(T > 0, "polarcub: no binary decode kernel for N=", N);
    auto xt = at::empty({(B + T - 1) / T, N, T, 2}, xy.options());
    check_rc(pcub_tile_pairs(xy.data_ptr<double>(), B, (int32_t)N, 2, T, xt.data_ptr<double>(), s), "pcub_tile_pairs");
    const size_t wsb = pcub_sc_decode_bin_workspace(B, n);
    auto ws = at::empty({(int64_t)std::max<size_t>(wsb, 16)}, u8);
    auto i32 = xy.options().dtype(at::kInt);
    auto iw = at::empty({std::max<int64_t>(1, (K + 31) / 32), B}, i32);
    auto xw = at::empty({(N + 31) / 32, B}, i32);
    check_rc(pcub_sc_decode_bin_tiled(xt.data_ptr<double>(), B, n, T,
                                      reinterpret_cast<const uint32_t*>(fm_words.data_ptr<int32_t>()),
                                      reinterpret_cast<const uint32_t*>(fv_words.data_ptr<int32_t>()), (int32_t)K,
                                      reinterpret_cast<uint32_t*>(iw.data_ptr<int32_t>()),
                                      reinterpret_cast<uint32_t*>(xw.data_ptr<int32_t>()), nullptr, ws.data_ptr(),
                                      (size_t)ws.numel(), s),
             "pcub_sc_decode_bin_tiled");
    return {unpack_words(iw, B, K, s), unpack_words(xw, B, N, s)};
}

std::tuple<at::Tensor, at::Tensor> sc_decode_bin_f64(const at::Tensor& xy_in, const at::Tensor& frozen_mask,
                                                     const at::Tensor& frozen_val) {
    check_xy_bin(xy_in);
    c10::OptionalDeviceGuard guard(xy_in.device());
    const int64_t N = xy_in.size(1);
    log2_exact(N);
    auto fm = mask_words(frozen_mask, N, xy_in.device());
    auto fv = mask_words(frozen_val, N, xy_in.device());
    return decode_bin_core(xy_in, fm.first, fv.first, N - fm.second);
}

void check_words(const at::Tensor& w, int64_t N, const at::Tensor& xy, const char* what) {
    TORCH_CHECK(w.device() == xy.device() && w.scalar_type() == at::kInt && w.is_contiguous() &&
                    w.numel() == std::max<int64_t>(1, (N + 31) / 32),
                "polarcub: ", what, " must be a contiguous int32 [ceil(N/32)] tensor on the xy device");
}

std::tuple<at::Tensor, at::Tensor> sc_decode_bin_words(const at::Tensor& xy_in, const at::Tensor& frozen_words,
                                                       const at::Tensor& frozen_val_words, int64_t K) {
    check_xy_bin(xy_in);
    c10::OptionalDeviceGuard guard(xy_in.device());
    const int64_t N = xy_in.size(1);
    log2_exact(N);
    check_words(frozen_words, N, xy_in, "frozen_words");
    check_words(frozen_val_words, N, xy_in, "frozen_val_words");
    TORCH_CHECK(K >= 0 && K <= N, "polarcub: K must be in [0, N], got ", K);
    return decode_bin_core(xy_in, frozen_words, frozen_val_words, K);
}

std::tuple<at::Tensor, at::Tensor> sc_decode_bin_words_meta(const at::Tensor& xy, const at::Tensor&,
                                                            const at::Tensor&, int64_t K) {
    auto u8 = xy.options().dtype(at::kByte);
    return {at::empty({xy.size(0), K}, u8), at::empty({xy.size(0), xy.size(1)}, u8)};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> sc_decode_bin_f64_leaf(const at::Tensor& xy_in,
                                                                      const at::Tensor& frozen_mask,
                                                                      const at::Tensor& frozen_val) {
    check_xy_bin(xy_in);
    c10::OptionalDeviceGuard guard(xy_in.device());
    const int64_t B = xy_in.size(0), N = xy_in.size(1);
    const int n = log2_exact(N);
    auto fm = mask_words(frozen_mask, N, xy_in.device());
    auto fv = mask_words(frozen_val, N, xy_in.device());
    const int64_t K = N - fm.second;
    auto u8 = xy_in.options().dtype(at::kByte);
    if (B == 0) return {at::empty({0, K}, u8), at::empty({0, N}, u8), at::empty({0, N, 2}, xy_in.options())};
    void* s = stream_of(xy_in);
    auto xy = xy_in.contiguous();
    auto xn = at::empty({N, B, 2}, xy.options());
    check_rc(pcub_transpose_pairs(xy.data_ptr<double>(), B, (int32_t)N, 2, xn.data_ptr<double>(), s),
             "pcub_transpose_pairs");
    const size_t wsb = pcub_sc_leaf_bin_workspace(B, n);
    auto ws = at::empty({(int64_t)std::max<size_t>(wsb, 16)}, u8);
    auto i32 = xy.options().dtype(at::kInt);
    auto iw = at::empty({std::max<int64_t>(1, (K + 31) / 32), B}, i32);
    auto xw = at::empty({(N + 31) / 32, B}, i32);
    auto leaf = at::empty({N, B}, xy.options());
    check_rc(pcub_sc_leaf_bin(xn.data_ptr<double>(), B, n,
                              reinterpret_cast<const uint32_t*>(fm.first.data_ptr<int32_t>()),
                              reinterpret_cast<const uint32_t*>(fv.first.data_ptr<int32_t>()), nullptr, (int32_t)K,
                              reinterpret_cast<uint32_t*>(iw.data_ptr<int32_t>()),
                              reinterpret_cast<uint32_t*>(xw.data_ptr<int32_t>()), leaf.data_ptr<double>(),
                              ws.data_ptr(), (size_t)ws.numel(), s),
             "pcub_sc_leaf_bin");
    auto marg = at::empty({N, B, 2}, xy.options());
    check_rc(pcub_leaf_marginals(leaf.data_ptr<double>(), N * B, marg.data_ptr<double>(), s), "pcub_leaf_marginals");
    return {unpack_words(iw, B, K, s), unpack_words(xw, B, N, s), marg.permute({1, 0, 2}).contiguous()};
}

at::Tensor mc_run(int64_t log2N, int64_t channel, double param, const at::Tensor& frozen_mask,
                  const at::Tensor& frozen_val, int64_t seed, int64_t cw_offset, int64_t count, int64_t chunk) {
    TORCH_CHECK(frozen_mask.is_cuda(), "polarcub: mc_run's frozen_mask must be a device tensor (it picks the GPU)");
    TORCH_CHECK(log2N >= 1 && log2N <= 20, "polarcub: mc_run needs 1 <= log2N <= 20, got ", log2N);
    TORCH_CHECK(channel == 0 || channel == 1, "polarcub: channel must be 0 (BI-AWGN) or 1 (BSC), got ", channel);
    TORCH_CHECK(seed >= 0 && cw_offset >= 0 && count >= 0 && chunk > 0,
                "polarcub: mc_run needs seed, cw_offset, count >= 0 and chunk > 0");
    const auto dev = frozen_mask.device();
    c10::OptionalDeviceGuard guard(dev);
    const int64_t N = int64_t(1) << log2N;
    auto fm = mask_words(frozen_mask, N, dev);
    auto fv = mask_words(frozen_val, N, dev);
    const int64_t K = N - fm.second;
    auto counters = at::zeros({4}, frozen_mask.options().dtype(at::kLong));
    if (count == 0) return counters;
    const int64_t ch = std::max<int64_t>(1, std::min(chunk, count));
    const size_t wsb = pcub_mc_run_bin_workspace(ch, (int32_t)log2N, (int32_t)K);
    TORCH_CHECK(wsb > 0, "polarcub: no Monte-Carlo pipeline for N=", N);
    auto ws = at::empty({(int64_t)wsb}, frozen_mask.options().dtype(at::kByte));
    check_rc(pcub_mc_run_bin((uint64_t)seed, cw_offset, count, (int32_t)log2N, (int32_t)channel, param,
                             reinterpret_cast<const uint32_t*>(fm.first.data_ptr<int32_t>()),
                             reinterpret_cast<const uint32_t*>(fv.first.data_ptr<int32_t>()), (int32_t)K, ch,
                             reinterpret_cast<uint64_t*>(counters.data_ptr<int64_t>()), ws.data_ptr(),
                             (size_t)ws.numel(), stream_of(frozen_mask)),
             "pcub_mc_run_bin");
    return counters;
}

std::tuple<at::Tensor, at::Tensor> sc_decode_qary_f64(int64_t q, const at::Tensor& xy_in,
                                                      const at::Tensor& frozen_mask) {
    TORCH_CHECK(q >= 2 && q <= 8, "polarcub: q must be in [2, 8], got ", q);
    TORCH_CHECK(xy_in.is_cuda() && xy_in.scalar_type() == at::kDouble && xy_in.dim() == 3 && xy_in.size(2) == q,
                "polarcub: xy must be a float64 [B, N, q] device tensor with q=", q);
    c10::OptionalDeviceGuard guard(xy_in.device());
    const int64_t B = xy_in.size(0), N = xy_in.size(1);
    const int n = log2_exact(N);
    TORCH_CHECK(frozen_mask.numel() == N, "polarcub: frozen mask has ", frozen_mask.numel(), " entries, expected N=", N);
    auto fz = frozen_mask.reshape({-1}).ne(0).to(at::kByte).to(xy_in.device()).contiguous();
    const int64_t K = N - fz.sum().item<int64_t>();
    auto u8 = xy_in.options().dtype(at::kByte);
    if (B == 0) return {at::empty({0, K}, u8), at::empty({0, N}, u8)};
    void* s = stream_of(xy_in);
    auto xy = xy_in.contiguous();
    const int T = pcub_sc_qary_tile((int32_t)q, n);
    TORCH_CHECK(T > 0, "polarcub: no q-ary decode kernel for q=", q, ", N=", N);
    auto xt = at::empty({(B + T - 1) / T, N, T, q}, xy.options());
    check_rc(pcub_tile_pairs(xy.data_ptr<double>(), B, (int32_t)N, (int32_t)q, T, xt.data_ptr<double>(), s),
             "pcub_tile_pairs");
    const size_t wsb = pcub_sc_decode_qary_workspace(B, n, (int32_t)q);
    auto ws = at::empty({(int64_t)std::max<size_t>(wsb, 16)}, u8);
    auto info = at::empty({std::max<int64_t>(1, K), B}, u8);
    auto xh = at::empty({N, B}, u8);
    check_rc(pcub_sc_decode_qary_tiled(xt.data_ptr<double>(), B, n, (int32_t)q, T, fz.data_ptr<uint8_t>(), (int32_t)K,
                                       info.data_ptr<uint8_t>(), xh.data_ptr<uint8_t>(), ws.data_ptr(),
                                       (size_t)ws.numel(), s),
             "pcub_sc_decode_qary_tiled");
    return {info.narrow(0, 0, K).t().contiguous(), xh.t().contiguous()};
}

at::Tensor polar_encode_bin(const at::Tensor& u_in) {
    TORCH_CHECK(u_in.is_cuda() && u_in.dim() == 2, "polarcub: u must be a [B, N] device tensor of bits");
    c10::OptionalDeviceGuard guard(u_in.device());
    const int64_t B = u_in.size(0), N = u_in.size(1);
    const int n = log2_exact(N);
    auto u = u_in.ne(0).to(at::kByte).contiguous();
    if (B == 0) return at::empty({0, N}, u.options());
    void* s = stream_of(u);
    const int64_t W = (N + 31) / 32;
    auto i32 = u.options().dtype(at::kInt);
    auto uw = at::empty({W, B}, i32);
    check_rc(pcub_pack_bits(u.data_ptr<uint8_t>(), B, (int32_t)N, reinterpret_cast<uint32_t*>(uw.data_ptr<int32_t>()),
                            s),
             "pcub_pack_bits");
    auto none = at::zeros({W}, i32);  // no frozen position: u is the whole decision vector (K = N)
    auto xw = at::empty({W, B}, i32);
    const auto* nw = reinterpret_cast<const uint32_t*>(none.data_ptr<int32_t>());
    check_rc(pcub_polar_encode_bin(reinterpret_cast<const uint32_t*>(uw.data_ptr<int32_t>()), B, n, nw, nw,
                                   (int32_t)N, reinterpret_cast<uint32_t*>(xw.data_ptr<int32_t>()), s),
             "pcub_polar_encode_bin");
    return unpack_words(xw, B, N, s);
}

}  // namespace

TORCH_LIBRARY(polarcub, m) {
    m.def("sc_decode_bin_f64(Tensor xy, Tensor frozen_mask, Tensor frozen_val) -> (Tensor, Tensor)");
    m.def("sc_decode_qary_f64(int q, Tensor xy, Tensor frozen_mask) -> (Tensor, Tensor)");
    m.def("polar_encode_bin(Tensor u) -> Tensor");
    m.def("sc_decode_bin_f64.leaf(Tensor xy, Tensor frozen_mask, Tensor frozen_val) -> (Tensor, Tensor, Tensor)");
    m.def("sc_decode_bin_words(Tensor xy, Tensor frozen_words, Tensor frozen_val_words, int K) -> (Tensor, Tensor)");
    m.def("mc_run(int log2N, int channel, float param, Tensor frozen_mask, Tensor frozen_val, int seed, "
          "int cw_offset, int count, int chunk=262144) -> Tensor");
}

TORCH_LIBRARY_IMPL(polarcub, CUDA, m) {
    m.impl("sc_decode_bin_f64", &sc_decode_bin_f64);
    m.impl("sc_decode_qary_f64", &sc_decode_qary_f64);
    m.impl("polar_encode_bin", &polar_encode_bin);
    m.impl("sc_decode_bin_f64.leaf", &sc_decode_bin_f64_leaf);
    m.impl("sc_decode_bin_words", &sc_decode_bin_words);
    m.impl("mc_run", &mc_run);
}

TORCH_LIBRARY_IMPL(polarcub, Meta, m) {
    m.impl("sc_decode_bin_words", &sc_decode_bin_words_meta);
}
