// Probe (diagnostic, GPU): can a stream wait in the device for a value that a
// worker thread writes behind work on another stream, while the main thread
// blocks in a synchronize?  Each case runs under a watchdog that ends the
// process (exit code 3) if it does not finish in time.
//
//   probe_wait_value <case>
//   case 0: main hipStreamSynchronize(waiting stream); worker writes the value
//   case 1: main hipDeviceSynchronize; worker writes the value
//   case 2: main hipDeviceSynchronize; worker launches kernels, event-syncs, then writes
//   case 3: case 2 with the worker's stream at normal priority
//   case 4: case 2, the value in device memory (hipMalloc) instead of signal memory
//   case 5: case 2 with the null stream waiting (torch's default current stream)
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unistd.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            _exit(2);                                                                           \
        }                                                                                       \
    } while (0)

__global__ void bump(float* x, int n, int reps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        for (int r = 0; r < reps; ++r) x[i] = x[i] * 0.999f + 1.0f;
}

int main(int argc, char** argv) {
    const int which = argc > 1 ? atoi(argv[1]) : 0;
    std::atomic<int> stage{0};
    std::thread dog([&] {
        for (int i = 0; i < 100; ++i) {
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
            if (stage.load() == 100) return;
        }
        printf("case %d: HANG (stage %d)\n", which, stage.load());
        fflush(stdout);
        _exit(3);
    });
    CK(hipSetDevice(0));
    int ok = 0;
    CK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("case %d: CanUseStreamWaitValue=%d\n", which, ok);
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t waiter, loop;
    if (which == 5) waiter = nullptr;
    else CK(hipStreamCreateWithFlags(&waiter, hipStreamNonBlocking));
    if (which == 3) CK(hipStreamCreateWithFlags(&loop, hipStreamNonBlocking));
    else CK(hipStreamCreateWithPriority(&loop, hipStreamNonBlocking, greatest));
    void* sig = nullptr;
    if (which == 4) CK(hipMalloc(&sig, 8));
    else CK(hipExtMallocWithFlags(&sig, 8, hipMallocSignalMemory));
    CK(hipStreamWriteValue64(loop, sig, 0, 0));
    CK(hipStreamSynchronize(loop));
    float* x = nullptr;
    const int n = 1 << 20;
    CK(hipMalloc(&x, n * sizeof(float)));
    CK(hipMemset(x, 0, n * sizeof(float)));
    float* y = nullptr;
    CK(hipMalloc(&y, sizeof(float)));
    CK(hipMemset(y, 0, sizeof(float)));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    stage = 1;
    CK(hipStreamWaitValue64(waiter, sig, 1, hipStreamWaitValueGte, ~0ull));
    hipLaunchKernelGGL(bump, dim3(1), dim3(1), 0, waiter, y, 1, 1);   // behind the wait
    CK(hipGetLastError());
    stage = 2;
    std::thread worker([&] {
        CK(hipSetDevice(0));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        if (which >= 2) {
            for (int b = 0; b < 8; ++b) {
                for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(bump, dim3(n / 256), dim3(256), 0, loop, x, n, 8);
                CK(hipGetLastError());
                CK(hipEventRecord(ev, loop));
                CK(hipEventSynchronize(ev));
            }
        }
        stage = 3;
        CK(hipStreamWriteValue64(loop, sig, 1, 0));
        CK(hipStreamSynchronize(loop));
        stage = 4;
    });
    const auto t0 = std::chrono::steady_clock::now();
    if (which == 0) CK(hipStreamSynchronize(waiter));
    else CK(hipDeviceSynchronize());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    worker.join();
    float hy = 0.f;
    CK(hipMemcpy(&hy, y, sizeof(float), hipMemcpyDeviceToHost));
    stage = 100;
    dog.join();
    printf("case %d: OK, main waited %.2f ms, kernel behind the wait ran: %s\n", which, ms, hy == 1.0f ? "yes" : "no");
    return 0;
}
