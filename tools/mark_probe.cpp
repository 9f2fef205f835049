// How a batch's completion can reach the host cheaply (the submission queue,
// shmr_amd/csrc/submit.cpp): per-call host cost of enqueueing each marker on
// an idle or a busy stream, and the time from enqueue (on an idle stream) to
// the host seeing it.
//   kernel      a one-wave kernel storing a sequence number to pinned host memory
//               (system-scope release; what the queue uses)
//   writevalue  hipStreamWriteValue64 of the number to the same word
//   event       hipEventRecord (completion seen by hipEventQuery polling)
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/_abx/mark_probe tools/mark_probe.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

__global__ void mark_kernel(uint64_t* word, uint64_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(word + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void busy_kernel(uint64_t* p, uint64_t n) {   // keeps the stream busy ~n iterations
    uint64_t x = threadIdx.x;
    for (uint64_t i = 0; i < n; ++i) x = x * 6364136223846793005ull + 1442695040888963407ull;
    if (x == 42) p[threadIdx.x] = x;   // never (keeps the loop)
}

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t* word = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&word), 64, hipHostMallocMapped));
    uint64_t* dword = nullptr;
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dword), word, 0));
    uint64_t* scratch = nullptr;
    CHECK(hipMalloc(reinterpret_cast<void**>(&scratch), 4096));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int N = 2000;
    uint64_t seq = 0;
    for (int mode = 0; mode < 3; ++mode) {
        const char* name = mode == 0 ? "kernel" : mode == 1 ? "writevalue" : "event";
        auto enqueue = [&](uint64_t v) {
            if (mode == 0) {
                hipLaunchKernelGGL(mark_kernel, dim3(1), dim3(64), 0, s, dword, v);
                CHECK(hipGetLastError());
            } else if (mode == 1) {
                CHECK(hipStreamWriteValue64(s, dword, v, 0));
            } else {
                CHECK(hipEventRecord(ev, s));
            }
        };
        auto seen = [&](uint64_t v) {
            if (mode == 2) return hipEventQuery(ev) == hipSuccess;
            return __atomic_load_n(word, __ATOMIC_ACQUIRE) >= v;
        };
        for (int i = 0; i < 100; ++i) enqueue(++seq);   // warm
        CHECK(hipStreamSynchronize(s));
        // enqueue cost, behind a busy kernel (nothing completes meanwhile)
        hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, s, scratch, 20000000ull);
        auto t0 = Clock::now();
        for (int i = 0; i < N; ++i) enqueue(++seq);
        auto t1 = Clock::now();
        CHECK(hipStreamSynchronize(s));
        const double enq_busy = us(t0, t1) / N;
        // enqueue cost on an idle stream, and enqueue -> host visibility
        std::vector<double> lat;
        double enq_idle = 0;
        for (int i = 0; i < 500; ++i) {
            const uint64_t v = ++seq;
            auto a = Clock::now();
            enqueue(v);
            auto b = Clock::now();
            while (!seen(v)) {
            }
            auto c = Clock::now();
            enq_idle += us(a, b);
            lat.push_back(us(a, c));
        }
        std::sort(lat.begin(), lat.end());
        std::printf("{\"marker\": \"%s\", \"enqueue_us_busy_stream\": %.2f, \"enqueue_us_idle\": %.2f, "
                    "\"visible_after_us_p50\": %.2f, \"p90\": %.2f}\n",
                    name, enq_busy, enq_idle / 500, lat[lat.size() / 2], lat[lat.size() * 9 / 10]);
        std::fflush(stdout);
    }
    return 0;
}
