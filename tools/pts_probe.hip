// Probe of one HIP runtime rule the IK stream test depends on (VERDICT r05 "next" 1): does
// hipDeviceSynchronize() on the main thread wait for work a host thread left on its per-thread default
// stream (hipStreamPerThread) after that thread has EXITED?  And does the thread's exit itself wait?
//
// A worker launches a bounded spin kernel (~0.3 s of wall clock, then one vector store of a flag) on
// hipStreamPerThread and records an event there, then either exits at once or stays alive until the
// main thread is done.  The main thread joins (or not), calls hipDeviceSynchronize() and reads the flag
// through a non-blocking stream (no implicit null-stream ordering), then waits on the event and reads
// again.
// Second question (round 6, from a failing test): may another thread order its own per-thread stream after
// that event with hipStreamWaitEvent once the recording thread has exited (its per-thread stream destroyed)?
// The waiting thread checks hipStreamIsCapturing on its stream and records / synchronizes an event of its own;
// the host-side alternative (hipEventQuery, hipEventSynchronize on the old event) is run beside it.
// Build: hipcc --offload-arch=gfx950 -O2 -o pts_probe tools/pts_probe.hip
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>

__global__ void spin_then_flag(int* flag, unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    flag[0] = 1;
}

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int read_flag(int* d, hipStream_t rd) {
    int h = -1;
    if (hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, rd) != hipSuccess) return -2;
    if (hipStreamSynchronize(rd) != hipSuccess) return -3;
    return h;
}

static int trial(bool exit_before_sync, int* flag, hipStream_t rd, unsigned long long ticks) {
    CK(hipMemset(flag, 0, sizeof(int)));
    CK(hipDeviceSynchronize());
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::atomic<int> launched{0}, release{0};
    double t_launch = 0, t_exit = 0;
    std::thread w([&] {
        (void)hipSetDevice(0);
        hipLaunchKernelGGL(spin_then_flag, dim3(1), dim3(1), 0, hipStreamPerThread, flag, ticks);
        (void)hipEventRecord(ev, hipStreamPerThread);
        t_launch = now_ms();
        launched = 1;
        while (!exit_before_sync && !release) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        t_exit = now_ms();
    });
    while (!launched) std::this_thread::sleep_for(std::chrono::microseconds(100));
    double t_join = 0;
    if (exit_before_sync) {
        w.join();
        t_join = now_ms();
    }
    CK(hipDeviceSynchronize());
    const double t_dsync = now_ms();
    const int after_dsync = read_flag(flag, rd);
    if (!exit_before_sync) {
        release = 1;
        w.join();
        t_join = now_ms();
    }
    CK(hipEventSynchronize(ev));
    const int after_event = read_flag(flag, rd);
    std::printf("%-34s join %.1f ms after launch (thread body ended %.1f ms after launch), "
                "hipDeviceSynchronize returned %.1f ms after launch: flag %d; after hipEventSynchronize: flag %d\n",
                exit_before_sync ? "worker exits before the sync:" : "worker alive during the sync:",
                t_join - t_launch, t_exit - t_launch, t_dsync - t_launch, after_dsync, after_event);
    CK(hipEventDestroy(ev));
    return 0;
}

static int wait_after_exit(bool device_wait, int* flag, unsigned long long ticks) {
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::thread a([&] {
        (void)hipSetDevice(0);
        hipLaunchKernelGGL(spin_then_flag, dim3(1), dim3(1), 0, hipStreamPerThread, flag, ticks / 30);
        (void)hipEventRecord(ev, hipStreamPerThread);
    });
    a.join();  // (its per-thread stream drained and destroyed at exit: see the first question)
    int r_wait = -1, r_cap = -1, r_rec = -1, r_sync = -1, r_q = -1;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    std::thread b([&] {
        (void)hipSetDevice(0);
        hipEvent_t mine;
        (void)hipEventCreateWithFlags(&mine, hipEventDisableTiming);
        if (device_wait) {
            r_wait = (int)hipStreamWaitEvent(hipStreamPerThread, ev, 0);
        } else {
            r_q = (int)hipEventQuery(ev);
            r_wait = (int)hipEventSynchronize(ev);
        }
        r_cap = (int)hipStreamIsCapturing(hipStreamPerThread, &cs);
        r_rec = (int)hipEventRecord(mine, hipStreamPerThread);
        r_sync = (int)hipEventSynchronize(mine);
        (void)hipStreamSynchronize(hipStreamPerThread);
        (void)hipEventDestroy(mine);
    });
    b.join();
    std::printf("%-44s wait %d, hipStreamIsCapturing %d (status %d), own event record %d, its synchronize %d%s\n",
                device_wait ? "other thread, hipStreamWaitEvent:" : "other thread, hipEventQuery + Synchronize:", r_wait,
                r_cap, (int)cs, r_rec, r_sync, device_wait ? "" : (" (query " + std::to_string(r_q) + ")").c_str());
    CK(hipEventDestroy(ev));
    return 0;
}

int main() {
    CK(hipSetDevice(0));
    int* flag = nullptr;
    CK(hipMalloc(&flag, sizeof(int)));
    hipStream_t rd;
    CK(hipStreamCreateWithFlags(&rd, hipStreamNonBlocking));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    if (khz <= 0 || khz > 10000000) khz = 100000;
    const unsigned long long ticks = 300ull * (unsigned long long)khz;  // 0.3 s of wall clock
    std::printf("wall clock %d kHz\n", khz);
    for (int rep = 0; rep < 3; ++rep) {
        if (trial(false, flag, rd, ticks)) return 1;
        if (trial(true, flag, rd, ticks)) return 1;
    }
    for (int rep = 0; rep < 2; ++rep) {
        if (wait_after_exit(false, flag, ticks)) return 1;
        if (wait_after_exit(true, flag, ticks)) return 1;
    }
    CK(hipStreamDestroy(rd));
    CK(hipFree(flag));
    return 0;
}
