// probe_resident.hip — feasibility of a resident step-server kernel: P one-wave blocks poll a request word each in
// device-mapped host memory (the step server's shared-memory slots), serve a row in place and publish done; host
// threads play the clients (write the row, post req, spin on done). Round-trip latency against a plain
// launch + synchronise per request. Every block exits on the quit word or on its own 20 s deadline (s_memrealtime).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/probe_resident.hip -o /tmp/probe_resident -lpthread
//   ./probe_resident [P] [N] [calls]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

struct alignas(64) Mail {
    uint32_t req, done, quit_seen, pad[13];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_resident(Mail* mail, const uint32_t* quit, double* rows, int N) {
    const int e = blockIdx.x, lane = threadIdx.x;
    Mail* m = mail + e;
    uint32_t served = __builtin_amdgcn_readfirstlane(ld_sys(&m->done));
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 20ull * 100000000ull;   // 100 MHz: 20 s
    double* row = rows + (size_t)e * 2 * N;
    for (uint32_t it = 0;; ++it) {
        const uint32_t r = __builtin_amdgcn_readfirstlane(ld_sys(&m->req));
        if (r == served) {
            if ((it & 15) == 0) {
                if (__builtin_amdgcn_readfirstlane(ld_sys(quit))) break;
                if (__builtin_amdgcn_s_memrealtime() > t_end) break;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        // the "step": every row negated and incremented by the request number (checked by the host)
        for (int i = lane; i < 2 * N; i += 64) row[i] = -row[i] + (double)r;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (lane == 0) st_sys(&m->done, r);
        served = r;
    }
    if (lane == 0) st_sys(&m->quit_seen, 1u);
}

__global__ void k_once(double* rows, int N, int e, uint32_t r) {
    double* row = rows + (size_t)e * 2 * N;
    for (int i = threadIdx.x; i < 2 * N; i += 64) row[i] = -row[i] + (double)r;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int P = argc > 1 ? std::atoi(argv[1]) : 16;
    const int N = argc > 2 ? std::atoi(argv[2]) : 181;
    const int calls = argc > 3 ? std::atoi(argv[3]) : 20000;
    const size_t mail_b = ((sizeof(Mail) * P + 4095) / 4096) * 4096, row_b = ((16ull * N * P + 4095) / 4096) * 4096;
    const size_t total = mail_b + row_b + 4096;
    // a shared mapping, as the step server's shm object (registered, device-mapped)
    uint8_t* base = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED) return 1;
    std::memset(base, 0, total);
    CK(hipHostRegister(base, total, hipHostRegisterMapped));
    uint8_t* dbase = nullptr;
    CK(hipHostGetDevicePointer((void**)&dbase, base, 0));
    Mail* mail = (Mail*)base;
    double* rows = (double*)(base + mail_b);
    uint32_t* quit = (uint32_t*)(base + mail_b + row_b);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // reference: a plain launch + synchronise per request (one client)
    {
        const int n = 2000;
        for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_once, 1, 64, 0, s, (double*)(dbase + mail_b), N, 0, 0u);
        CK(hipStreamSynchronize(s));
        const double t0 = now_us();
        for (int i = 0; i < n; ++i) {
            hipLaunchKernelGGL(k_once, 1, 64, 0, s, (double*)(dbase + mail_b), N, 0, 0u);
            CK(hipStreamSynchronize(s));
        }
        std::printf("{\"kind\": \"launch_sync\", \"us_per_call\": %.2f}\n", (now_us() - t0) / n);
    }
    std::memset(rows, 0, 16ull * N * P);
    hipLaunchKernelGGL(k_resident, P, 64, 0, s, (Mail*)dbase, (const uint32_t*)(dbase + mail_b + row_b),
                       (double*)(dbase + mail_b), N);
    CK(hipGetLastError());
    for (int T : {1, P}) {
        std::vector<std::thread> th;
        std::vector<double> us(T, 0.0);
        std::atomic<int> bad{0};
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t]() {
                Mail* m = mail + t;
                double* row = rows + (size_t)t * 2 * N;
                double t0 = 0.0;
                const int warm = 200;
                for (int i = 0; i < calls + warm; ++i) {
                    if (i == warm) t0 = now_us();
                    const uint32_t r = __atomic_load_n(&m->req, __ATOMIC_RELAXED) + 1u;
                    for (int k = 0; k < 2 * N; ++k) row[k] = (double)k;
                    __atomic_store_n(&m->req, r, __ATOMIC_RELEASE);
                    const double tw = now_us();
                    while (__atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != r) {
                        __builtin_ia32_pause();
                        if (now_us() - tw > 2e6) { bad++; return; }   // 2 s: no answer
                    }
                    for (int k = 0; k < 2 * N; ++k)
                        if (row[k] != -(double)k + (double)r) { bad++; break; }
                }
                us[t] = (now_us() - t0) / calls;
            });
        for (auto& x : th) x.join();
        double avg = 0;
        for (double v : us) avg += v / T;
        std::printf("{\"kind\": \"resident\", \"clients\": %d, \"N\": %d, \"us_per_call\": %.2f, \"calls_per_s\": %.0f, \"bad\": %d}\n",
                    T, N, avg, T / avg * 1e6, bad.load());
        if (bad.load()) break;
    }
    __atomic_store_n(quit, 1u, __ATOMIC_RELEASE);
    const double tq = now_us();
    CK(hipStreamSynchronize(s));
    int seen = 0;
    for (int e = 0; e < P; ++e) seen += mail[e].quit_seen ? 1 : 0;
    std::printf("{\"kind\": \"quit\", \"blocks_exited\": %d, \"of\": %d, \"us\": %.1f}\n", seen, P, now_us() - tq);
    CK(hipHostUnregister(base));
    munmap(base, total);
    return 0;
}
