// Store-pattern probe for the x6r (16x16x32 form) epilogue: 256 workgroups x 4 waves, each
// wave storing its 128 pixels x 32 fp32 channels (16 KB) of a 256 x 64 output item, 16 items
// per workgroup (inc.3's shape: 4096 items of 256 px x 64 co, NHWC rows of 256 B), all
// workgroups in lockstep as in the conv.  Patterns (16 dwordx4 stores per wave and item):
//   A: the MFMA fragment layout -- lane (g, l) writes pixel l's channels 16nt+4g..+3: each
//      instruction = 16 pixels x 64 B (16 half lines)
//   B: pixel-major rows -- lane L writes pixel (L>>3) of an 8-pixel group, channels
//      4(L&7)..+3: each instruction = 8 pixels x 128 B (8 whole lines)
//   C/D: A/B with non-temporal stores
// Prints the kernel time per pattern (median of 20) and the per-item store time per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.cpp -o exp/store_probe && exp/store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ void __launch_bounds__(256) store_kernel(float* out, int items_per_wg, float seed) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
    const int g = lane >> 4, l16 = lane & 15;
    f32x4 v = {seed + lane, seed - lane, seed * lane, seed + w};
    for (int it = 0; it < items_per_wg; ++it) {
        const size_t item = (size_t)it * gridDim.x + blockIdx.x;
        float* base = out + (item * 256 + wm * 128) * 64 + wn * 32;  // pixel-major, 64 ch / pixel
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float* p;
            if constexpr (PAT == 0 || PAT == 2) {
                const int mt = i >> 1, nt = i & 1;
                p = base + (size_t)(mt * 16 + l16) * 64 + nt * 16 + 4 * g;
            } else {
                p = base + (size_t)(i * 8 + (lane >> 3)) * 64 + 4 * (lane & 7);
            }
            v.x += 1.f;
            if constexpr (PAT >= 2)
                __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
            else
                *reinterpret_cast<f32x4*>(p) = v;
        }
    }
}

// the same 64 KB per workgroup and item stored by NW waves (64/NW dwordx4 per wave), 16 lanes x
// 16 B per 256-B pixel row segment as pattern A
template <int NW>
__global__ void __launch_bounds__(64 * NW) store_waves_kernel(float* out, int items_per_wg, float seed) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    f32x4 v = {seed + lane, seed - lane, seed * lane, seed + w};
    constexpr int PER = 64 / NW;
    for (int it = 0; it < items_per_wg; ++it) {
        const size_t item = (size_t)it * gridDim.x + blockIdx.x;
        float* base = out + item * 256 * 64;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int ins = w * PER + i;  // 64 instructions of 1 KiB: 4 pixels x 256 B each
            float* p = base + (size_t)(ins * 4 + (lane >> 4)) * 64 + 4 * (lane & 15);
            v.x += 1.f;
            *reinterpret_cast<f32x4*>(p) = v;
        }
    }
}

template <int NW>
static double time_waves(float* out, int wgs, int items, hipEvent_t e0, hipEvent_t e1) {
    std::vector<float> ts;
    for (int r = 0; r < 20; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(store_waves_kernel<NW>, dim3(wgs), dim3(64 * NW), 0, 0, out, items, 1.f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

// the conv-like regime: every workgroup "computes" (a dependent FMA chain of `spin` steps per
// wave) between its items' store bursts, optionally with staggered phases (workgroup w starts
// w % 8 / 8 of an item late), 4 storing waves, pattern A / B / W (whole 1-KiB runs: 4 pixels x
// all 64 channels per instruction); do_store = 0 times the compute alone
template <int PAT>
__global__ void __launch_bounds__(256) conv_like_kernel(float* out, int items_per_wg, int spin,
                                                        int stagger, int do_store) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
    const int g = lane >> 4, l16 = lane & 15;
    float x = 1.f + lane * 1e-3f;
    const int off = stagger ? spin * (int)(blockIdx.x % 8) / 8 : 0;
    for (int i = 0; i < off; ++i) x = fmaf(x, 0.999f, 0.5f);
    f32x4 v = {x, x + 1.f, x + 2.f, x + 3.f};
    for (int it = 0; it < items_per_wg; ++it) {
        for (int i = 0; i < spin; ++i) x = fmaf(x, 0.999f, 0.5f);
        v.x += x;
        if (!do_store) continue;
        const size_t item = (size_t)it * gridDim.x + blockIdx.x;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float* p;
            if constexpr (PAT == 0) {
                float* base = out + (item * 256 + wm * 128) * 64 + wn * 32;
                p = base + (size_t)((i >> 1) * 16 + l16) * 64 + (i & 1) * 16 + 4 * g;
            } else if constexpr (PAT == 1) {
                float* base = out + (item * 256 + wm * 128) * 64 + wn * 32;
                p = base + (size_t)(i * 8 + (lane >> 3)) * 64 + 4 * (lane & 7);
            } else {
                p = out + (item * 256 + (size_t)(w * 16 + i) * 4 + (lane >> 4)) * 64 + 4 * (lane & 15);
            }
            *reinterpret_cast<f32x4*>(p) = v;
        }
    }
    if (x == 12345.f) out[0] = x;
}

constexpr int SPIN = 600;

int main() {
    const int wgs = 256, items = 16;
    const size_t n = (size_t)wgs * items * 256 * 64;
    float* out;
    if (hipMalloc(&out, n * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[4] = {"A fragment (16 px x 64 B)", "B rows (8 px x 128 B)", "C = A non-temporal",
                            "D = B non-temporal"};
    // per-CU limit or chip-wide bandwidth: the same per-workgroup work on 256, 128, 64, 32 CUs
    for (int ng : {32}) {  // pattern B (8 px x 128 B: whole lines, not contiguous) per CU
        std::vector<float> ts;
        for (int r = 0; r < 20; ++r) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(store_kernel<1>, dim3(ng), dim3(256), 0, 0, out, items, 1.f);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double ms = ts[ts.size() / 2];
        printf("B on %3d workgroups: %8.1f us  %7.0f ns per item per CU\n", ng, ms * 1e3, ms * 1e6 / items);
    }
    for (int ng : {256, 128, 64, 32}) {
        std::vector<float> ts;
        for (int r = 0; r < 20; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(store_kernel<0>, dim3(ng), dim3(256), 0, 0, out, items, 1.f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double ms = ts[ts.size() / 2];
        printf("A on %3d workgroups: %8.1f us  %6.2f TB/s  %7.0f ns per item per CU\n", ng, ms * 1e3,
               (double)ng * items * 65536 / (ms * 1e-3) / 1e12, ms * 1e6 / items);
    }
    for (int rep = 0; rep < 2; ++rep) {
        for (int pat = 0; pat < 4; ++pat) {
            std::vector<float> ts;
            for (int r = 0; r < 20; ++r) {
                hipEventRecord(e0);
                if (pat == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(wgs), dim3(256), 0, 0, out, items, 1.f);
                if (pat == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(wgs), dim3(256), 0, 0, out, items, 1.f);
                if (pat == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(wgs), dim3(256), 0, 0, out, items, 1.f);
                if (pat == 3) hipLaunchKernelGGL(store_kernel<3>, dim3(wgs), dim3(256), 0, 0, out, items, 1.f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0.f;
                hipEventElapsedTime(&ms, e0, e1);
                ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            const double ms = ts[ts.size() / 2];
            const double bytes = (double)n * sizeof(float);
            if (rep == 1)
                printf("%-28s %8.1f us  %6.2f TB/s  %7.0f ns per item per CU\n", names[pat], ms * 1e3,
                       bytes / (ms * 1e-3) / 1e12, ms * 1e6 / items);
        }
    }
    for (int wgs2 : {256, 32}) {
        const double t[5] = {time_waves<1>(out, wgs2, items, e0, e1), time_waves<2>(out, wgs2, items, e0, e1),
                             time_waves<4>(out, wgs2, items, e0, e1), time_waves<8>(out, wgs2, items, e0, e1),
                             time_waves<16>(out, wgs2, items, e0, e1)};
        for (int i = 0; i < 5; ++i)
            printf("%2d storing waves, %3d workgroups (whole 1-KiB runs): %7.1f us  %7.0f ns per item per CU\n",
                   1 << i, wgs2, t[i] * 1e3, t[i] * 1e6 / items);
    }
    // conv-like: ~10 us of compute per item (SPIN), 16 items, all 256 CUs
    for (int stagger : {0, 1}) {
        for (int pat = 0; pat < 3; ++pat) {
            double t[2];
            for (int ds = 0; ds < 2; ++ds) {
                std::vector<float> ts;
                for (int r = 0; r < 7; ++r) {
                    (void)hipEventRecord(e0);
                    if (pat == 0) hipLaunchKernelGGL(conv_like_kernel<0>, dim3(wgs), dim3(256), 0, 0, out, items, SPIN, stagger, ds);
                    if (pat == 1) hipLaunchKernelGGL(conv_like_kernel<1>, dim3(wgs), dim3(256), 0, 0, out, items, SPIN, stagger, ds);
                    if (pat == 2) hipLaunchKernelGGL(conv_like_kernel<2>, dim3(wgs), dim3(256), 0, 0, out, items, SPIN, stagger, ds);
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms = 0.f;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                t[ds] = ts[ts.size() / 2];
            }
            printf("conv-like %s, pattern %c: %8.1f us with stores, %8.1f us without: %6.0f ns per item\n",
                   stagger ? "staggered" : "lockstep ", "ABW"[pat], t[1] * 1e3, t[0] * 1e3,
                   (t[1] - t[0]) * 1e6 / items);
        }
    }
    if (hipGetLastError() != hipSuccess) return 2;
    hipFree(out);
    return 0;
}
