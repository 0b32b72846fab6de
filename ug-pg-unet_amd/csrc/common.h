// Shared helpers for the libugpg HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/ugpg.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace ugpg {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return UGPG_ERR_LAUNCH;
    }
    return UGPG_OK;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid size for memory-bound grid-stride kernels (cap ~8 blocks per CU).
inline unsigned stream_grid(int64_t work, int block = 256) {
    int64_t g = cdiv(work, block);
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    return (unsigned)g;
}

__device__ __forceinline__ float act_apply(float v, const float* sc, const float* sh, int c) {
    return sc ? fmaxf(fmaf(v, sc[c], sh[c]), 0.0f) : v;
}

__device__ __forceinline__ f32x4 act_apply4(f32x4 v, const float* sc, const float* sh, int c) {
    if (sc) {
        f32x4 s = *reinterpret_cast<const f32x4*>(sc + c);
        f32x4 h = *reinterpret_cast<const f32x4*>(sh + c);
        v.x = fmaxf(fmaf(v.x, s.x, h.x), 0.0f);
        v.y = fmaxf(fmaf(v.y, s.y, h.y), 0.0f);
        v.z = fmaxf(fmaf(v.z, s.z, h.z), 0.0f);
        v.w = fmaxf(fmaf(v.w, s.w, h.w), 0.0f);
    }
    return v;
}

// Lazy-activation coefficients of 4 channels held in registers: conv kernels load
// them together with the data they will transform (a load at LDS-store time would
// stall the whole block on a global round trip).
struct Act4 {
    f32x4 s, h;
};
__device__ __forceinline__ Act4 act_load4(const float* sc, const float* sh, int c) {
    Act4 r;
    if (sc) {
        r.s = *reinterpret_cast<const f32x4*>(sc + c);
        r.h = *reinterpret_cast<const f32x4*>(sh + c);
    } else {
        r.s = f32x4{1.f, 1.f, 1.f, 1.f};
        r.h = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    return r;
}
// on == false: identity (no BatchNorm+ReLU on this operand)
__device__ __forceinline__ f32x4 act_reg4(f32x4 v, const Act4& a, bool on) {
    if (on) {
        v.x = fmaxf(fmaf(v.x, a.s.x, a.h.x), 0.0f);
        v.y = fmaxf(fmaf(v.y, a.s.y, a.h.y), 0.0f);
        v.z = fmaxf(fmaf(v.z, a.s.z, a.h.z), 0.0f);
        v.w = fmaxf(fmaf(v.w, a.s.w, a.h.w), 0.0f);
    }
    return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// align_corners=True source index/weight exactly as ATen computes them in fp32
// (area_pixel_compute_scale + guard_index_and_lambda): scale = (in-1)/(out-1),
// src = scale*o, i0 = min(floor(src), in-1), l1 = clamp(src-i0, 0, 1).
__device__ __forceinline__ void ac_index(int o, int in, int out, int& i0, int& i1, float& l0,
                                         float& l1) {
    if (in == out) {
        i0 = i1 = o;
        l0 = 1.0f;
        l1 = 0.0f;
        return;
    }
    float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.0f;
    float src = scale * (float)o;
    int f = (int)floorf(src);
    i0 = f < in - 1 ? f : in - 1;
    float l = src - (float)i0;
    l1 = fminf(fmaxf(l, 0.0f), 1.0f);
    i1 = i0 + (i0 < in - 1 ? 1 : 0);
    l0 = 1.0f - l1;
}

}  // namespace ugpg
