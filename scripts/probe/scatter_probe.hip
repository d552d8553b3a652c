// Probe (not product code): throughput of scattered 16-B global loads on gfx950 — how many
// lane-requests per second the vector memory path sustains when every lane of a wave-instruction
// hits a different line, against coalesced loads.  Prints one JSON line per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned u32;
typedef unsigned long long u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4u;

__device__ __forceinline__ u64 mix(u64 x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }

// MODE 0: per lane K loads, each a random 16-B-aligned address (a different line per lane)
// MODE 1: per lane K/4 random 64-B pieces, 4 consecutive 16-B loads each
// MODE 2: per wave K random 1-KiB blocks, lane l loads bytes 16l.. (coalesced)
// MODE 3: like 0 but byte-unaligned addresses
// DEP: loads of a lane depend on the previous one (a chain) instead of independent batches of 4
template <int MODE, int DEP>
__global__ __launch_bounds__(256) void k(const unsigned char* __restrict__ buf, u64 mask_lines, int K, u32* out) {
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 wid = gid >> 6;
    const u32 lane = threadIdx.x & 63;
    u32 acc = 0;
    u64 h = mix(gid * 0x9E3779B97F4A7C15ull + 1);
    for (int i = 0; i < K; i += 4) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            u64 a;
            if (MODE == 0) a = (mix(h + i + j + (DEP ? acc : 0)) & mask_lines) * 16;
            else if (MODE == 3) a = (mix(h + i + j + (DEP ? acc : 0)) & mask_lines) * 16 + ((h >> 7) & 15);
            else if (MODE == 1) a = (mix(h + i + (DEP ? acc : 0)) & (mask_lines >> 2)) * 64 + 16 * j;
            else a = (mix(wid * 0x9E3779B97F4A7C15ull + i + j + (DEP ? acc : 0)) & (mask_lines >> 6)) * 1024 + 16 * lane;
            v[j] = MODE == 3 ? *(const u32x4u*)(buf + a) : *(const u32x4*)(buf + a);
            if (DEP) acc += v[j].x & 1;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int MODE, int DEP>
void run(const char* name, const unsigned char* buf, u64 bytes, int blocks, int K, u32* out) {
    u64 mask = (bytes / 16) - 1;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k<MODE, DEP>), dim3(blocks), dim3(256), 0, 0, buf, mask, K, out);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL((k<MODE, DEP>), dim3(blocks), dim3(256), 0, 0, buf, mask, K, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
    double lanereq = (double)blocks * 256 * K;
    printf("{\"variant\": \"%s\", \"buf_mb\": %llu, \"ms\": %.4f, \"Greq_per_s\": %.2f, \"useful_TBps\": %.3f}\n", name,
           bytes >> 20, ms, lanereq / ms / 1e6, lanereq * 16 / ms / 1e9);
}

int main() {
    const u64 big = 4ull << 30, small = 2ull << 20;
    unsigned char* buf; u32* out;
    hipMalloc(&buf, big); hipMalloc(&out, 4);
    hipMemset(buf, 1, big);
    const int K = 64;
    for (int blocks : {256 * 4, 256 * 8}) {
        printf("# blocks %d (x256 threads)\n", blocks);
        run<2, 0>("coalesced_1k", buf, big, blocks, K, out);
        run<0, 0>("scatter16", buf, big, blocks, K, out);
        run<3, 0>("scatter16_unaligned", buf, big, blocks, K, out);
        run<1, 0>("scatter64_4x16", buf, big, blocks, K, out);
        run<0, 0>("scatter16_L2", buf, small, blocks, K, out);
        run<3, 0>("scatter16u_L2", buf, small, blocks, K, out);
        run<2, 0>("coalesced_1k_L2", buf, small, blocks, K, out);
        run<0, 1>("scatter16_chain", buf, big, blocks, K, out);
        run<0, 1>("scatter16_chain_L2", buf, small, blocks, K, out);
    }
    hipFree(buf);
    return 0;
}
