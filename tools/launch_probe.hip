// launch_probe.hip — what a dependent kernel boundary costs on this runtime,
// and what the device loop's launch path adds to it (round 6).
//
// Every case enqueues R launches of one kernel shape behind a busy kernel
// (a bounded spin on the 100 MHz wall clock), so the host has queued them all
// before the GPU reaches the first: the event pair around them then measures
// the GPU's own per-launch cost, not the host's launch rate.  The host's
// enqueue cost per launch is reported beside it (wall time of the launch
// calls).  One JSON line per case on stdout.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip
//   tools/launch_probe [R]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

// bounded spin: `ticks` of the 100 MHz constant clock (every wave exits)
__global__ void busy_kernel(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void empty_kernel() {}

struct Big {
    double v[64];  // 512-byte by-value argument, like LoopCfg
};
__global__ void bigarg_kernel(Big b, int* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[3] == -1.0) out[0] = 1;
}

// the loop kernels' prologue: read the control word, return if set
__global__ void ctl_kernel(const int* __restrict__ ctl, int* __restrict__ out) {
    if (*ctl) return;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = 1;
}

// ...and every thread stores one float (dirty lines left for the boundary)
__global__ void ctl_store_kernel(const int* __restrict__ ctl, float* __restrict__ out, int n) {
    if (*ctl) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)i;
}

// a kernel argument pointing into pinned host memory, read by lane 0
__global__ void hostread_kernel(const int* __restrict__ hflag, int* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && *hflag == 12345) out[2] = 1;
}
// a host-memory pointer passed but never dereferenced
__global__ void hostptr_kernel(const int* __restrict__ hflag, int* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && hflag == nullptr) out[2] = 1;
}

// the finalize pattern: one ticket per block behind a release, last block reads
__global__ void ticket_kernel(unsigned* __restrict__ ticket, double* __restrict__ out, int nv) {
    __shared__ int last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&out[blockIdx.x], 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        const unsigned o = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = o == (unsigned)(nv - 1);
    }
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Res {
    double gpu_us, host_us;
};

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
Res run_case(hipStream_t s, int R, F&& launch, long long busy_ticks = 300000 /* 3 ms */) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // warm (module load, kernarg pool)
    for (int i = 0; i < 8; ++i) launch(i);
    CK(hipStreamSynchronize(s));
    hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, s, busy_ticks);
    CK(hipEventRecord(e0, s));
    const double h0 = now_us();
    for (int i = 0; i < R; ++i) launch(i);
    const double h1 = now_us();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    Res r{ms * 1e3 / R, (h1 - h0) / R};
    // the busy kernel must outlast the enqueue, else the GPU waited for the host
    if ((h1 - h0) > busy_ticks / 100.0 * 0.9) r.gpu_us = -r.gpu_us;  // (flagged: host-bound)
    return r;
}

static void emit(const char* name, const char* note, Res r) {
    std::printf("{\"case\": \"%s\", \"gpu_us_per_launch\": %.3f, \"host_us_per_launch\": %.3f, \"note\": \"%s\"}\n",
                name, r.gpu_us, r.host_us, note);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 400;
    CK(hipSetDevice(0));
    hipStream_t s, sp_hi, sp_lo, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&sp_hi, hipStreamNonBlocking, greatest));
    CK(hipStreamCreateWithPriority(&sp_lo, hipStreamNonBlocking, least));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int *d_ctl, *d_out, *h_flag;
    float* d_f;
    double* d_d;
    unsigned* d_ticket;
    const int nf = 3907 * 256;
    CK(hipMalloc(&d_ctl, 64));
    CK(hipMemset(d_ctl, 0, 64));
    CK(hipMalloc(&d_out, 64));
    CK(hipMalloc(&d_f, sizeof(float) * nf));
    CK(hipMalloc(&d_d, sizeof(double) * 64));
    CK(hipMalloc(&d_ticket, 64));
    CK(hipMemset(d_ticket, 0, 64));
    CK(hipHostMalloc((void**)&h_flag, 4096, hipHostMallocDefault));
    std::memset(h_flag, 0, 4096);
    void* h_stat;
    CK(hipHostMalloc(&h_stat, 8192, hipHostMallocDefault));
    hipEvent_t done_ev;
    CK(hipEventCreateWithFlags(&done_ev, hipEventDisableTiming));
    CK(hipEventRecord(done_ev, s2));
    CK(hipDeviceSynchronize());

    const char* kd = std::getenv("HIP_FORCE_DEV_KERNARG");
    std::printf("{\"env\": {\"HIP_FORCE_DEV_KERNARG\": \"%s\"}, \"R\": %d}\n", kd ? kd : "(unset)", R);

    emit("empty_1x64", "", run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); }));
    emit("empty_64x256", "", run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(256), 0, s); }));
    emit("empty_256x256", "", run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s); }));
    emit("empty_512x256", "", run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(256), 0, s); }));
    emit("empty_3907x256", "the C3 match grid",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(3907), dim3(256), 0, s); }));
    emit("empty_15625x64", "the cold tile grid",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(15625), dim3(64), 0, s); }));
    Big b{};
    emit("bigarg_1x64", "512 B by value",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(bigarg_kernel, dim3(1), dim3(64), 0, s, b, d_out); }));
    emit("bigarg_3907x256", "512 B by value",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(bigarg_kernel, dim3(3907), dim3(256), 0, s, b, d_out); }));
    emit("ctl_1x64", "ctl word read",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(ctl_kernel, dim3(1), dim3(64), 0, s, d_ctl, d_out); }));
    emit("ctl_3907x256", "ctl word read",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(ctl_kernel, dim3(3907), dim3(256), 0, s, d_ctl, d_out); }));
    emit("ctl_store_3907x256", "4 MB stored",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(ctl_store_kernel, dim3(3907), dim3(256), 0, s, d_ctl, d_f, nf); }));
    emit("hostread_1x64", "pinned host word read",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(hostread_kernel, dim3(1), dim3(64), 0, s, h_flag, d_out); }));
    emit("hostptr_1x64", "pinned host pointer, not read",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(hostptr_kernel, dim3(1), dim3(64), 0, s, h_flag, d_out); }));
    emit("ticket_32x256", "finalize ticket",
         run_case(s, R, [&](int) { hipLaunchKernelGGL(ticket_kernel, dim3(32), dim3(256), 0, s, d_ticket, d_d, 32); }));
    emit("ext_1x64", "hipExtLaunchKernelGGL, no events", run_case(s, R, [&](int) {
             hipExtLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr, nullptr, 0);
         }));
    emit("ext_3907x256", "hipExtLaunchKernelGGL, no events", run_case(s, R, [&](int) {
             hipExtLaunchKernelGGL(empty_kernel, dim3(3907), dim3(256), 0, s, nullptr, nullptr, 0);
         }));
    emit("prio_hi_1x64", "greatest priority stream",
         run_case(sp_hi, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, sp_hi); }));
    emit("prio_lo_1x64", "least priority stream",
         run_case(sp_lo, R, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, sp_lo); }));
    emit("waitev_1x64", "hipStreamWaitEvent on a completed event before each", run_case(s, R, [&](int) {
             (void)hipStreamWaitEvent(s, done_ev, 0);
             hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
         }));
    emit("d2h_every8_1x64", "7.5 KB D2H to pinned + event after every 8th", run_case(s, R, [&](int i) {
             hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
             if ((i & 7) == 7) {
                 (void)hipMemcpyAsync(h_stat, d_f, 7680, hipMemcpyDeviceToHost, s);
                 (void)hipEventRecord(done_ev, s);
             }
         }));
    emit("record_each_1x64", "hipEventRecord (timing) after each", run_case(s, R, [&](int) {
             static hipEvent_t ev = nullptr;
             if (!ev) (void)hipEventCreate(&ev);
             hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
             (void)hipEventRecord(ev, s);
         }));
    // the same four-launch shape as a C3 iteration, empty bodies
    emit("iter4_empty", "3907x256, 64x256, 512x256, 32x256 (per launch)", run_case(s, R, [&](int i) {
             switch (i & 3) {
                 case 0: hipLaunchKernelGGL(ctl_kernel, dim3(3907), dim3(256), 0, s, d_ctl, d_out); break;
                 case 1: hipLaunchKernelGGL(ctl_kernel, dim3(64), dim3(256), 0, s, d_ctl, d_out); break;
                 case 2: hipLaunchKernelGGL(ctl_kernel, dim3(512), dim3(256), 0, s, d_ctl, d_out); break;
                 default: hipLaunchKernelGGL(ticket_kernel, dim3(32), dim3(256), 0, s, d_ticket, d_d, 32); break;
             }
         }));
    // a captured graph of 64 empty launches, replayed
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const int reps = std::max(1, R / 64);
        Res r = run_case(s, reps, [&](int) { (void)hipGraphLaunch(ge, s); });
        r.gpu_us /= 64;
        r.host_us /= 64;
        emit("graph64_1x64", "per kernel node", r);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipDeviceSynchronize());
    return 0;
}
