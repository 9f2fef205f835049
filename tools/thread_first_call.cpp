// What a thread's FIRST HIP calls cost (r06 s14: the queue's first launch in a
// rep, made by a freshly created submitting thread while it held the
// queue's launcher flag, kept the GPU idle ~120-190 us).  Each of 8 new
// threads times its first and second hipGetDevice, hipSetDevice,
// hipThreadExchangeStreamCaptureMode, kernel launch on a shared stream and
// hipEventRecord; one JSON line per thread.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/_abx/thread_first_call tools/thread_first_call.cpp -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void nop_kernel(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 0;   // never true
}

using Clock = std::chrono::steady_clock;

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 1;
    hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, s, nullptr);
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    for (int t = 0; t < 8; ++t) {
        std::thread([&, t] {
            double us[2][5];
            for (int rep = 0; rep < 2; ++rep) {
                auto a = Clock::now();
                int d = -1;
                (void)hipGetDevice(&d);
                auto b = Clock::now();
                (void)hipSetDevice(0);
                auto c = Clock::now();
                hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
                (void)hipThreadExchangeStreamCaptureMode(&mode);
                (void)hipThreadExchangeStreamCaptureMode(&mode);
                auto e = Clock::now();
                hipLaunchKernelGGL(nop_kernel, dim3(128), dim3(256), 0, s, nullptr);
                auto f = Clock::now();
                (void)hipEventRecord(ev, s);
                auto g = Clock::now();
                auto u = [](Clock::time_point x, Clock::time_point y) {
                    return std::chrono::duration<double, std::micro>(y - x).count();
                };
                us[rep][0] = u(a, b);
                us[rep][1] = u(b, c);
                us[rep][2] = u(c, e);
                us[rep][3] = u(e, f);
                us[rep][4] = u(f, g);
            }
            std::printf("{\"thread\": %d, \"first_us\": {\"getdevice\": %.1f, \"setdevice\": %.1f, \"capture_mode_x2\": %.1f, "
                        "\"launch\": %.1f, \"event_record\": %.1f}, \"second_us\": {\"getdevice\": %.1f, \"setdevice\": %.1f, "
                        "\"capture_mode_x2\": %.1f, \"launch\": %.1f, \"event_record\": %.1f}}\n",
                        t, us[0][0], us[0][1], us[0][2], us[0][3], us[0][4], us[1][0], us[1][1], us[1][2], us[1][3],
                        us[1][4]);
            std::fflush(stdout);
        }).join();
    }
    return hipStreamSynchronize(s) == hipSuccess ? 0 : 1;
}
