// scl.hip -- q-ary SCL / Fast-SSC list decoding on gfx950 (scl_body.h), one lane per codeword,
// + C-ABI.  QaryPolarEncoderDecoder.listDecode (QaryPolarEncoderDecoder.py:118-227, 403-820).
//
// Each lane walks the (frozen-mask-determined) recursion of its codeword with its list of up to
// L paths in a per-slot slab (slot-minor, so the lanes of a wave, all at the same point of the
// same recursion, touch consecutive words).  The recursion is a loop over an explicit frame
// stack (scl_run), so the kernel has a fixed private segment and no dynamic stack: the launch
// never depends on the device's per-thread stack limit, and the library never changes it.
// (A wave-per-codeword layout with lanes over positions was measured in round 5 at 0.66 k vs
// 1.65 k cw/s at q = 4, N = 4096, L = 32 and removed)
// List decoding is a host-side tool in the reference
// (the IR simulation); the kernel batches it, it is not the SC throughput path.
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "scl_body.h"

using namespace pcub;

namespace {

constexpr int kSclBlock = 64;

__global__ __launch_bounds__(kSclBlock) void k_scl(SclArgs A) {
    const long long slot = (long long)blockIdx.x * kSclBlock + threadIdx.x;
    const long long ntiles = (A.B + kSclBlock - 1) / kSclBlock;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * kSclBlock + threadIdx.x;
        const bool valid = cw < A.B;
        scl_decode_cw(A, valid ? cw : A.B - 1, slot, valid);
    }
}

bool scl_args_ok(int64_t B, int32_t q, int32_t log2N, int32_t L, int32_t K) {
    return B >= 0 && q >= 2 && q <= 8 && log2N >= 0 && log2N <= 12 && L >= 1 && L <= 64 && K >= 0 &&
           K <= (1 << log2N);
}

// workgroups of a launch: 8 a CU (64 codewords each)
long long scl_grid(long long B) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    const long long ntiles = (B + kSclBlock - 1) / kSclBlock;
    const long long g = (long long)cus * 8;
    return ntiles < g ? ntiles : g;
}

// slots (codewords in flight) of a launch: kSclBlock per workgroup
long long scl_slots(long long B) { return scl_grid(B) * kSclBlock; }

size_t scl_slot_bytes(int32_t q, int32_t log2N, int32_t L, int32_t K) {
    SclLayout Y;
    Y.init(log2N, q, L, K);
    return (size_t)Y.ncells * 8 + (size_t)Y.nbytes;
}

}  // namespace

extern "C" size_t pcub_scl_qary_workspace(int64_t B, int32_t q, int32_t log2N, int32_t L, int32_t K) {
    if (B <= 0 || !scl_args_ok(B, q, log2N, L, K)) return 0;
    return (size_t)scl_slots(B) * scl_slot_bytes(q, log2N, L, K) + 16;
}

namespace {

int launch_scl(bool lg, const double* xy, int64_t B, int32_t q, int32_t log2N, int32_t L, const uint8_t* frozen,
               const uint8_t* frozen_vals, int32_t nF, const uint8_t* actual, int32_t K, uint8_t* out_info,
               double* out_prob, int32_t* out_size, double* out_actual, void* workspace, size_t workspace_bytes,
               void* stream) {
    if (!scl_args_ok(B, q, log2N, L, K) || !frozen || nF < 0 || nF + K != (1 << log2N)) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!xy || (nF > 0 && !frozen_vals) || !out_info || !out_prob || !out_size || !workspace) return PCUB_EINVAL;
    if (actual && !out_actual) return PCUB_EINVAL;
    long long g = scl_grid(B);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kSclBlock * scl_slot_bytes(q, log2N, L, K);
    if ((size_t)g * per_block > workspace_bytes) g = (long long)(workspace_bytes / per_block);
    if (g <= 0) return PCUB_EINVAL;
    SclLayout Y;
    Y.init(log2N, q, L, K);
    SclArgs A;
    A.xy = xy;
    A.B = B;
    A.n = log2N;
    A.q = q;
    A.L = L;
    A.K = K;
    A.frozen = frozen;
    A.fvals = frozen_vals;
    A.nF = nF;
    A.actual = actual;
    A.out_info = out_info;
    A.out_prob = out_prob;
    A.out_size = (int*)out_size;
    A.out_actual = out_actual;
    A.log = lg ? 1 : 0;
    A.ns = g * kSclBlock;
    A.cells = (double*)workspace;
    A.bytes = (uint8_t*)workspace + (size_t)Y.ncells * 8 * (size_t)A.ns;
    hipLaunchKernelGGL(k_scl, dim3((unsigned)g), dim3(kSclBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" int pcub_scl_qary(const double* xy, int64_t B, int32_t q, int32_t log2N, int32_t L,
                             const uint8_t* frozen, const uint8_t* frozen_vals, int32_t nF, const uint8_t* actual,
                             int32_t K, uint8_t* out_info, double* out_prob, int32_t* out_size, double* out_actual,
                             void* workspace, size_t workspace_bytes, void* stream) {
    return launch_scl(false, xy, B, q, log2N, L, frozen, frozen_vals, nF, actual, K, out_info, out_prob, out_size,
                      out_actual, workspace, workspace_bytes, stream);
}

// use_log=True: xy holds log-probabilities; out_prob / out_actual are log-domain metrics
extern "C" int pcub_scl_qary_log(const double* xy, int64_t B, int32_t q, int32_t log2N, int32_t L,
                                 const uint8_t* frozen, const uint8_t* frozen_vals, int32_t nF, const uint8_t* actual,
                                 int32_t K, uint8_t* out_info, double* out_prob, int32_t* out_size, double* out_actual,
                                 void* workspace, size_t workspace_bytes, void* stream) {
    return launch_scl(true, xy, B, q, log2N, L, frozen, frozen_vals, nF, actual, K, out_info, out_prob, out_size,
                      out_actual, workspace, workspace_bytes, stream);
}
