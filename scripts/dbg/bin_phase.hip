// Diagnostic build (not the product): where the binary decode kernel's time goes.  A copy of
// decode_codeword (sc_bin_sched.h) for the split-level variant 26 shape, with s_memtime stamps
// around the non-final chain passes, the final pass into registers/LDS, hl_run and the rest
// (re-encoded bit combines, info bits, x_hat), summed per wave.  Inputs: the all-zero codeword over
// BI-AWGN at Eb/N0 = 2 dB (rate 1/2), the bench's Bhattacharyya frozen set, frozen values 0.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I polarcub_amd/csrc -I include \
//         scripts/dbg/bin_phase.hip -o scripts/dbg/bin_phase && ./scripts/dbg/bin_phase [log2B]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "sc_bin_kern.h"

using namespace pcub;



namespace {

struct Acc {
    unsigned long long pass = 0, fin = 0, hl = 0, rest = 0;
    unsigned long long fk[4] = {0, 0, 0, 0}, hk[4] = {0, 0, 0, 0};  // final pass / hl_run time by chain k
};

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }

template <int S, int G, int PF, int PF1 = -1>
__device__ void decode_timed(const BinArgs& A, long long cw, int j, int lane, long long slot, bool store,
                             uint32_t* ylds, long long ystride, double* hl, Acc& T) {
    constexpr bool LDS = false, YL = true, HL = true, CR = false;
    constexpr int NT = 1;
    constexpr int SR = 2 * S;
    constexpr int s = 6;
    constexpr int g = (G == 4) ? 2 : 3;
    using W = SubWin<SR, G>;
    constexpr int NW = W::NW;
    constexpr int RR = 2;
    constexpr bool NS = false;
    const int n = A.n;
    const int nv = n - g;
    const int Nv = 1 << nv;
    const int D = nv - s;
    const long long ns = A.nslots;
    const long long B = A.B;
    const long long rowbase = root_base(A, cw) + 2 * (long long)bitrev((uint32_t)j, n - 1) * root_stride(A);
    const double2* in = A.xy + rowbase;
    double2* scr = A.scratch + slot;
    uint32_t* Y = ylds;
    const long long ys = ystride;
    LevelMap lm;
    lm.scr = scr;
    lm.ns = ns;
    lm.Nv = Nv;
    lm.D = D;
    lm.last = Lvl{nullptr, 0};
    Lvl lastlv;
    uint64_t acc = 0;
    int nacc = 0;
    int infow = 0;
    unsigned long long t0 = now();
    for (int k = 0; k < (1 << D); ++k) {
        in = launder(in);
        scr = launder(scr);
        lm.scr = scr;
        lastlv = lm.get(D - 1);
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        const int e0 = A.ef[k];
        int a = d0 - 1;
        bool fg = (k != 0);
        Chain c;
        c.in = in;
        c.lin = 0;
        c.inc = nullptr;
        c.B = root_stride(A);
        c.nv = nv;
        c.Y = Y;
        c.ns = ys;
        uint64_t fm[NW], fv[NW], ub[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int us = k * SR * G + 64 * w;
            const int uw = us >> 5;
            fm[w] = (uint64_t)A.fmask[uw] | ((uint64_t)A.fmask[uw + 1] << 32);
            fv[w] = (uint64_t)A.fval[uw] | ((uint64_t)A.fval[uw + 1] << 32);
            ub[w] = 0;
        }
        uint64_t y;
        unsigned long long t1 = now();
        T.rest += t1 - t0;
        t0 = t1;
        if (e0 <= D - 1) {
            int Tl = e0 - 1 - a;
            while (Tl > 0) {
                const int F = Tl >= 3 ? 3 : Tl;
                c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
                c.ystart = (k >> (D - a)) << (nv - a);
                const int La = Nv >> a;
                if (F == 3) dispatch_pass<3, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else if (F == 2) dispatch_pass<2, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else dispatch_pass<1, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                a += F;
                Tl -= F;
                fg = false;
            }
            y = hl_frozen<S, G>(ub, fv, j);
            t1 = now();
            T.pass += t1 - t0;
            t0 = t1;
        } else {
            int Tl = D - a;
            const int Ffin = final_levels<LDS>(Tl);
            while (Tl > Ffin) {
                const int F = (Tl - Ffin) >= 3 ? 3 : (Tl - Ffin);
                c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
                c.ystart = (k >> (D - a)) << (nv - a);
                const int La = Nv >> a;
                if (F == 3) dispatch_pass<3, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else if (F == 2) dispatch_pass<2, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else dispatch_pass<1, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                a += F;
                Tl -= F;
                fg = false;
            }
            t1 = now();
            T.pass += t1 - t0;
            t0 = t1;
            constexpr int HS = S;
            double v[SR - HS];
            c.ystart = (k >> (D - a)) << (nv - a);
            if (Ffin == 2) {
                c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
                dispatch_final<SR, 2, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, a == 0, hl);
            } else if (a > 0) {
                c.src = lastlv;
                dispatch_final<SR, 1, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, false, hl);
            } else {
                dispatch_final<SR, 1, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, true, hl);
            }
            t1 = now();
            T.fin += t1 - t0;
            T.fk[k & 3] += t1 - t0;
            t0 = t1;
            if (e0 == D) y = hl_frozen<S, G>(ub, fv, j);
            else y = hl_run<S, G>(hl, v, ub, fm, fv, lane);
            t1 = now();
            T.hl += t1 - t0;
            T.hk[k & 3] += t1 - t0;
            t0 = t1;
        }
        const int lstart = k * SR;
        uint32_t* yw = Y + (long long)(lstart >> 5) * ys;
        sty<YL>(yw, (uint32_t)y);
        sty<YL>(yw + ys, (uint32_t)(y >> 32));
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            for (uint64_t im = ~fm[w]; im != 0ull; im &= im - 1ull) {
                const int q = __builtin_ctzll(im);
                acc |= ((ub[w] >> q) & 1ull) << nacc;
                if (++nacc == 32) {
                    if (store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
                    acc = 0;
                    nacc = 0;
                    ++infow;
                }
            }
        }
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = Nv >> d;
            const int Wc = Lc >> 5;
            uint32_t* base = Y + (long long)((k >> (D - d + 1)) * (2 * Wc)) * ys;
            for (int w = 0; w < Wc; ++w)
                sty<YL>(base + (long long)w * ys, ldy<YL>(base + (long long)w * ys) ^ ldy<YL>(base + (long long)(w + Wc) * ys));
        }
    }
    if (nacc && store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
    if (A.xhat && store) {
        const int seg = (int)bitrev((uint32_t)j, g);
        const int Wn = Nv >> 5;
        for (int w = 0; w < Wn; ++w) {
            uint32_t o = 0;
            for (int t = 0; t < 32; ++t) {
                const uint32_t p = bitrev((uint32_t)(32 * w + t), nv);
                o |= ((ldy<YL>(Y + (long long)(p >> 5) * ys) >> (p & 31u)) & 1u) << t;
            }
            A.xhat[(long long)(seg * Wn + w) * B + cw] = o;
        }
    }
    T.rest += now() - t0;
}

template <int PF1>
__global__ __launch_bounds__(kBinBlock, 2) void k_timed(BinArgs A, unsigned long long* out) {
    extern __shared__ double2 lds_last[];
    constexpr int S = 32, G = 4;
    constexpr int LDS2 = S / 2 * kBinBlock;
    constexpr int CWB = kBinBlock / G;
    const long long slot = (long long)blockIdx.x * kBinBlock + threadIdx.x;
    const int j = threadIdx.x & (G - 1);
    const int lane = threadIdx.x & 63;
    const long long ntiles = (A.B + CWB - 1) / CWB;
    Acc T;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * CWB + threadIdx.x / G;
        const bool valid = cw < A.B;
        decode_timed<S, G, 2, PF1>(A, valid ? cw : A.B - 1, j, lane, slot, valid,
                                       (uint32_t*)(lds_last + LDS2) + threadIdx.x, kBinBlock,
                                       (double*)lds_last + threadIdx.x, T);
    }
    if (lane == 0) {
        const long long wv = (long long)blockIdx.x * (kBinBlock / 64) + threadIdx.x / 64;
        out[wv * 12 + 0] = T.pass;
        out[wv * 12 + 1] = T.fin;
        out[wv * 12 + 2] = T.hl;
        out[wv * 12 + 3] = T.rest;
        for (int i = 0; i < 4; ++i) {
            out[wv * 12 + 4 + i] = T.fk[i];
            out[wv * 12 + 8 + i] = T.hk[i];
        }
    }
}

// the library's decode_codeword, variant 26's shape with prefetch distances PF / PF1
template <int PF, int PF1>
__global__ __launch_bounds__(kBinBlock, 2) void k_real(BinArgs A, unsigned long long*) {
    extern __shared__ double2 lds_last[];
    constexpr int S = 32, G = 4;
    constexpr int LDS2 = S / 2 * kBinBlock;
    constexpr int CWB = kBinBlock / G;
    const long long slot = (long long)blockIdx.x * kBinBlock + threadIdx.x;
    const int j = threadIdx.x & (G - 1);
    const int lane = threadIdx.x & 63;
    const long long ntiles = (A.B + CWB - 1) / CWB;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * CWB + threadIdx.x / G;
        const bool valid = cw < A.B;
        decode_codeword<S, G, false, 1, true, true, PF, false, PF1>(
            A, valid ? cw : A.B - 1, j, lane, slot, valid, Lvl{nullptr, 0}, (uint32_t*)(lds_last + LDS2) + threadIdx.x,
            kBinBlock, (double*)lds_last + threadIdx.x);
    }
}

// all-zero codeword over BPSK/AWGN: y = 1 + sigma * N(0,1) (a counter-hash Box-Muller), joint rows
__global__ void k_inputs(double2* xy, long long count, double sigma2, long long B, int N, int tile) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const long long r = i / B, cw = i % B;  // element (row r, codeword cw) of the [N][B] layout
    const long long dst = tile ? (cw / tile) * ((long long)N * tile) + r * tile + cw % tile : i;
    unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 27;
    h *= 0x94D049BB133111EBull;
    h ^= h >> 31;
    const double u1 = ((h >> 11) + 1.0) * (1.0 / 9007199254740993.0);
    unsigned long long h2 = h * 0xD1B54A32D192ED03ull + 1;
    h2 ^= h2 >> 29;
    const double u2 = (h2 >> 11) * (1.0 / 9007199254740992.0);
    const double z = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
    const double y = 1.0 + sqrt(sigma2) * z;
    const double c = 0.5 / sqrt(2.0 * M_PI * sigma2);
    xy[dst] = double2{c * exp(-(y - 1.0) * (y - 1.0) / (2.0 * sigma2)), c * exp(-(y + 1.0) * (y + 1.0) / (2.0 * sigma2))};
}

__global__ void k_ef(const uint32_t* fmask, int D, int SU, uint8_t* ef) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < (1 << D)) ef[k] = (uint8_t)first_frozen_depth(fmask, k, D, SU);
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef void (*Kern)(BinArgs, unsigned long long*);

std::vector<uint32_t> g_ref;  // info words of the first run (bit-exactness check of the others)

void run(const char* name, Kern k, bool stamped, BinArgs A, size_t lds, long long grid, unsigned long long* dout,
         int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemset(A.info, 0, (size_t)(1 << A.n) / 64 * A.B * 4));
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kBinBlock), lds, 0, A, dout);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> info((size_t)(1 << A.n) / 64 * A.B);
    CK(hipMemcpy(info.data(), A.info, info.size() * 4, hipMemcpyDeviceToHost));
    const char* same = "";
    if (g_ref.empty()) g_ref = info;
    else same = (info == g_ref) ? " [info = first run]" : " [INFO DIFFERS]";
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kBinBlock), lds, 0, A, dout);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-34s %7.3f ms/launch %7.2f M cw/s%s", name, ms, A.B / (ms * 1e3), same);
    if (stamped) {
        const long long nw = grid * (kBinBlock / 64);
        std::vector<unsigned long long> h(nw * 12);
        CK(hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost));
        double s[12] = {};
        for (long long w = 0; w < nw; ++w)
            for (int i = 0; i < 12; ++i) s[i] += (double)h[w * 12 + i];
        const double tot = s[0] + s[1] + s[2] + s[3];
        printf("  shares: passes %.3f final %.3f hl_run %.3f rest %.3f | final by k %.3f %.3f %.3f %.3f | hl by k %.3f %.3f "
               "%.3f %.3f",
               s[0] / tot, s[1] / tot, s[2] / tot, s[3] / tot, s[4] / tot, s[5] / tot, s[6] / tot, s[7] / tot,
               s[8] / tot, s[9] / tot, s[10] / tot, s[11] / tot);
    }
    printf("\n");
    fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const int lb = argc > 1 ? atoi(argv[1]) : 20;
    const long long B = 1LL << lb;
    const int n = 10, N = 1 << n, K = N / 2, G = 4, SR = 64;
    const double sigma2 = 1.0 / (2.0 * 0.5 * pow(10.0, 0.2));
    // frozen = the N - K least reliable by the Bhattacharyya recursion (bench.py / construction.py)
    std::vector<double> z(1, exp(-1.0 / (2.0 * sigma2)));
    for (int l = 0; l < n; ++l) {
        std::vector<double> nz(2 * z.size());
        for (size_t i = 0; i < z.size(); ++i) {
            nz[2 * i] = 2 * z[i] - z[i] * z[i];
            nz[2 * i + 1] = z[i] * z[i];
        }
        z.swap(nz);
    }
    std::vector<int> order(N);
    for (int i = 0; i < N; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return z[a] < z[b]; });
    std::vector<uint32_t> fm(N / 32, 0xffffffffu), fv(N / 32, 0u);
    for (int i = 0; i < K; ++i) fm[order[i] >> 5] &= ~(1u << (order[i] & 31));
    const int nv = n - 2, Nv = 1 << nv, D = nv - 6;
    int occ = 2, cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const long long ntiles = (B + 63) / 64;
    const long long grid = std::min(ntiles, (long long)cus * occ);
    const long long nslots = grid * kBinBlock;
    double2* xy;
    CK(hipMalloc(&xy, (size_t)B * N * sizeof(double2)));
    hipLaunchKernelGGL(k_inputs, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, 0, xy, B * N, sigma2, B, N, 0);
    uint32_t *dfm, *dfv, *info, *xh;
    CK(hipMalloc(&dfm, N / 8));
    CK(hipMalloc(&dfv, N / 8));
    CK(hipMemcpy(dfm, fm.data(), N / 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dfv, fv.data(), N / 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&info, (size_t)(K / 32) * B * 4));
    CK(hipMalloc(&xh, (size_t)(N / 32) * B * 4));
    double2* scr;
    CK(hipMalloc(&scr, (size_t)nslots * (Nv / 2 - SR) * sizeof(double2) + 16));
    uint8_t* ef;
    CK(hipMalloc(&ef, 256));
    hipLaunchKernelGGL(k_ef, dim3(1), dim3(256), 0, 0, dfm, D, SR * G, ef);
    unsigned long long* dout;
    CK(hipMalloc(&dout, (size_t)grid * 4 * 12 * 8));
    BinArgs A;
    A.xy = xy;
    A.xc = nullptr;
    A.B = B;
    A.n = n;
    A.fmask = dfm;
    A.fval = dfv;
    A.info = info;
    A.xhat = xh;
    A.uout = nullptr;
    A.scratch = scr;
    A.ybits = nullptr;
    A.nslots = nslots;
    A.ef = ef;
    A.tile = 0;
    const size_t lds = (size_t)32 * kBinBlock * 8 + (size_t)kBinBlock * (Nv / 32) * 4;
    const int reps = 5;
    const int only = argc > 2 ? atoi(argv[2]) : -1;  // run one configuration (profilers)
    struct Cfg {
        const char* name;
        Kern k;
        bool stamped;
    };
    const Cfg cfgs[] = {
        {"v26 (PF 2)", k_real<2, -1>, false},
        {"stamped v26", k_timed<-1>, true},
    };
    for (int i = 0; i < (int)(sizeof(cfgs) / sizeof(cfgs[0])); ++i)
        if (only < 0 || only == i) run(cfgs[i].name, cfgs[i].k, cfgs[i].stamped, A, lds, grid, dout, reps);
    // the same codewords with the root in [B/16][N][16] tiles (one wave's 16 codewords contiguous)
    hipLaunchKernelGGL(k_inputs, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, 0, xy, B * N, sigma2, B, N, 16);
    A.tile = 16;
    run("v26, root in 16-codeword tiles", k_real<2, -1>, false, A, lds, grid, dout, reps);
    run("stamped, tiles", k_timed<-1>, true, A, lds, grid, dout, 2);
    return 0;
}
