// Calibration only (never part of libkartdiff): rocPRIM's library radix sort of 32-bit key + 32-bit
// value pairs on the same shapes kd_sort_side sorts (C3: 100M keys, 27 varying bits), timed with HIP
// events — a reference point for k_sort_pass's achieved bandwidth on this GPU.
#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
    const int bits = argc > 2 ? atoi(argv[2]) : 27;
    std::vector<unsigned> hk(n), hv(n);
    unsigned long long x = 88172645463325252ull;
    for (size_t i = 0; i < n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        hk[i] = (unsigned)(x & ((1ull << bits) - 1));
        hv[i] = (unsigned)i;
    }
    unsigned *ki, *ko, *vi, *vo;
    CK(hipMalloc(&ki, n * 4)); CK(hipMalloc(&ko, n * 4)); CK(hipMalloc(&vi, n * 4)); CK(hipMalloc(&vo, n * 4));
    CK(hipMemcpy(ki, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(vi, hv.data(), n * 4, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, ki, ko, vi, vo, n, 0, bits));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 2; w++) CK(rocprim::radix_sort_pairs(tmp, tb, ki, ko, vi, vo, n, 0, bits));
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs(tmp, tb, ki, ko, vi, vo, n, 0, bits));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned> ok(n);
    CK(hipMemcpy(ok.data(), ko, n * 4, hipMemcpyDeviceToHost));
    bool sorted = true;
    for (size_t i = 1; i < n; i++) sorted &= ok[i - 1] <= ok[i];
    printf("{\"what\": \"rocprim::radix_sort_pairs u32 key + u32 value\", \"n\": %zu, \"bits\": %d, \"ms_per_sort\": %.4f, "
           "\"sorted\": %s, \"temp_bytes\": %zu}\n", n, bits, ms / reps, sorted ? "true" : "false", tb);
    return 0;
}
