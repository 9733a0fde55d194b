// pmx_robust.hip — the scale estimators of RobustOutlierFilter
// (OutlierFiltersImpl.cpp:494-534) on the device.
//
//   mad   sqrt(Matches::getMedianAbsDeviation()) (Matches.cpp:88-122): the
//         median of the finite distances (exact index size / 2, one radix
//         select), the absolute deviations from it (launch_abs_dev), their
//         median (a second select) — pmx_capi.hip sequences them;
//   std   sqrt(Matches::getStandardDeviation()) (Matches.cpp:124-129): over
//         ALL k x N distances (+inf included, as the reference), mean then
//         the corrected second moment; sums of T values in fp64, the rest in T;
//   berg  1.9 sqrt(median) at the first iteration, then
//         0.85 (scale - target) + target (the convergence toward the target).
// The scale stays on the device (a T value in a double slot per chain
// position); the weighted reductions read it (pmx_internal.h robust_weight).
#include "pmx_internal.h"

namespace pmx {

// ctl (device loop, may be null): every kernel returns at once once the loop
// has stopped or stalled, as the other kernels of an iteration
template <typename T>
__global__ void abs_dev_kernel(const T* __restrict__ d, int64_t n, const SelectState* __restrict__ st,
                               T* __restrict__ dev, const LoopCtl* __restrict__ ctl) {
    if (ctl && ctl->done) return;
    const T med = (T)st->limit;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T v = d[i];
        dev[i] = v != (T)__builtin_huge_val() ? fabs(v - med) : v;
    }
}

template <typename T>
void launch_abs_dev(const T* d, int64_t n, const SelectState* st, T* dev, const LoopCtl* ctl, hipStream_t s) {
    if (n <= 0) return;
    int64_t g = (n + 1023) / 1024;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(abs_dev_kernel<T>, dim3((unsigned)g), dim3(256), 0, s, d, n, st, dev, ctl);
}

// pass 0: sum d; pass 1: sum (d - mean)^2, mean = (T)(sum / n_total) (T
// arithmetic per term; n_total: every rank's count, the sum being all-reduced)
template <typename T>
__global__ __launch_bounds__(256) void moment_kernel(const T* __restrict__ d, int64_t n, int pass,
                                                     const double* __restrict__ sum, double* __restrict__ partials,
                                                     int64_t n_total, const LoopCtl* __restrict__ ctl) {
    __shared__ double red[4];
    if (ctl && ctl->done) return;
    const T mean = pass ? (T)(*sum / (double)n_total) : (T)0;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T v = d[i];
        if (pass) {
            const T c = v - mean;
            acc += (double)(c * c);
        } else {
            acc += (double)v;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

template <typename T>
void launch_moment(const T* d, int64_t n, int pass, const double* sum, double* partials, int64_t n_total,
                   const LoopCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(moment_kernel<T>, dim3(kRedBlocks), dim3(256), 0, s, d, n, pass, sum, partials, n_total, ctl);
}

template <typename T>
__global__ void robust_scale_kernel(int mode, const SelectState* __restrict__ st, const double* __restrict__ sums,
                                    int64_t n, double target, double* __restrict__ scale,
                                    const LoopCtl* __restrict__ ctl) {
    if (threadIdx.x != 0 || (ctl && ctl->done)) return;
    T sc = (T)*scale;
    switch (mode) {
    case kRSNone: sc = (T)1; break;
    case kRSMad: sc = sqrt((T)st->limit); break;
    case kRSStd: {  // sqrt(sqrt(sum (d - mean)^2 / (size - 1)))
        const T var = (T)sums[1] / (T)(n - 1);
        sc = sqrt(sqrt(var));
        break;
    }
    case kRSBergFirst: sc = (T)(1.9 * (double)sqrt((T)st->limit)); break;
    case kRSBergNext: {
        const T rate = (T)0.85, tg = (T)target;  // CONVERGENCE_RATE (OutlierFiltersImpl.cpp:523)
        sc = rate * (sc - tg) + tg;
        break;
    }
    default: break;  // keep the previous iteration's scale
    }
    *scale = (double)sc;
}

template <typename T>
void launch_robust_scale(int mode, const SelectState* st, const double* sums, int64_t n, double target,
                         double* scale, const LoopCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(robust_scale_kernel<T>, dim3(1), dim3(64), 0, s, mode, st, sums, n, target, scale, ctl);
}

#define PMX_ROBUST_INST(T)                                                                                        \
    template void launch_abs_dev<T>(const T*, int64_t, const SelectState*, T*, const LoopCtl*, hipStream_t);      \
    template void launch_moment<T>(const T*, int64_t, int, const double*, double*, int64_t, const LoopCtl*,       \
                                   hipStream_t);                                                                  \
    template void launch_robust_scale<T>(int, const SelectState*, const double*, int64_t, double, double*,       \
                                         const LoopCtl*, hipStream_t);
PMX_ROBUST_INST(float)
PMX_ROBUST_INST(double)
#undef PMX_ROBUST_INST

}  // namespace pmx
