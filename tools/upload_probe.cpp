// Host -> device upload rates for the setup path (development probe):
// pageable hipMemcpyAsync, pinned DMA, pinned staging filled by T host
// threads, hipHostRegister, and the host's sequential reference mean.
// build: hipcc -O2 -std=c++17 tools/upload_probe.cpp -o tools/upload_probe -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x)                                                       \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                               \
        }                                                           \
    } while (0)

int main() {
    const size_t bytes = 28u << 20;  // 1M float4 points + 1M float3 normals
    std::vector<char> src(bytes);
    for (size_t i = 0; i < bytes; ++i) src[i] = (char)(i * 7);
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto best = [](auto f) {
        double b = 1e9;
        for (int r = 0; r < 5; ++r) {
            const double t = now();
            f();
            b = std::min(b, now() - t);
        }
        return b;
    };
    double t = best([&] {
        (void)hipMemcpyAsync(d, src.data(), bytes, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
    });
    std::printf("pageable hipMemcpyAsync 28 MB: %.3f ms (%.1f GB/s)\n", t * 1e3, bytes / t / 1e9);
    void* h = nullptr;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    std::memcpy(h, src.data(), bytes);
    t = best([&] {
        (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
    });
    std::printf("pinned DMA 28 MB: %.3f ms (%.1f GB/s)\n", t * 1e3, bytes / t / 1e9);
    for (int T : {1, 2, 4, 8, 16}) {
        t = best([&] {
            std::vector<std::thread> th;
            const size_t per = (bytes + T - 1) / T;
            for (int k = 0; k < T; ++k)
                th.emplace_back([&, k] {
                    const size_t a = k * per, b = std::min(bytes, a + per);
                    if (a < b) std::memcpy((char*)h + a, src.data() + a, b - a);
                });
            for (auto& x : th) x.join();
        });
        std::printf("host memcpy into pinned, %2d threads: %.3f ms (%.1f GB/s)\n", T, t * 1e3, bytes / t / 1e9);
    }
    // staged pipeline: chunks of C bytes, T threads fill chunk i while chunk i-1 DMAs
    for (size_t C : {(size_t)2 << 20, (size_t)4 << 20, (size_t)8 << 20})
        for (int T : {4, 8}) {
            hipEvent_t ev[2];
            (void)hipEventCreateWithFlags(&ev[0], hipEventDisableTiming);
            (void)hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
            t = best([&] {
                const size_t nch = (bytes + C - 1) / C;
                for (size_t i = 0; i < nch; ++i) {
                    const int b = (int)(i & 1);
                    char* stg = (char*)h + b * C;
                    (void)hipEventSynchronize(ev[b]);
                    const size_t off = i * C, len = std::min(C, bytes - off);
                    std::vector<std::thread> th;
                    const size_t per = (len + T - 1) / T;
                    for (int k = 0; k < T; ++k)
                        th.emplace_back([&, k] {
                            const size_t a = k * per, e = std::min(len, a + per);
                            if (a < e) std::memcpy(stg + a, src.data() + off + a, e - a);
                        });
                    for (auto& x : th) x.join();
                    (void)hipMemcpyAsync((char*)d + off, stg, len, hipMemcpyHostToDevice, s);
                    (void)hipEventRecord(ev[b], s);
                }
                (void)hipStreamSynchronize(s);
            });
            std::printf("staged %zu MB chunks, %d threads: %.3f ms (%.1f GB/s)\n", C >> 20, T, t * 1e3, bytes / t / 1e9);
        }
    t = best([&] {
        (void)hipHostRegister(src.data(), bytes, hipHostRegisterDefault);
        void* dp = nullptr;
        (void)hipHostGetDevicePointer(&dp, src.data(), 0);
        (void)hipMemcpyAsync(d, src.data(), bytes, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
        (void)hipHostUnregister(src.data());
    });
    std::printf("hipHostRegister + DMA + unregister 28 MB: %.3f ms\n", t * 1e3);
    // the host's sequential reference mean over 1M float4 points
    const float* f = (const float*)src.data();
    volatile float sink = 0;
    t = best([&] {
        float a = 0, b = 0, c = 0;
        for (size_t j = 0; j < (1u << 20); ++j) {
            a = a + f[j * 4];
            b = b + f[j * 4 + 1];
            c = c + f[j * 4 + 2];
        }
        sink = a + b + c;
    });
    std::printf("sequential mean, 1M points: %.3f ms\n", t * 1e3);
    (void)sink;
    return 0;
}
