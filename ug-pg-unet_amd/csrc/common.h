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

// 4 consecutive bf16 (8 bytes) widened to fp32 (exact)
__device__ __forceinline__ f32x4 ld4_bf16(const __bf16* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                 __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
}
// An NHWC activation stored in fp32 or (the bf16 arithmetic's storage, ugpg_src_t
// data_bf16) in bf16: exactly one of f / h is set.  The choice is uniform per kernel, so
// the branch in ld4 costs a scalar test.
struct YRef {
    const float* f;
    const __bf16* h;
    __device__ __forceinline__ f32x4 ld4(size_t off) const {
        return f ? *reinterpret_cast<const f32x4*>(f + off) : ld4_bf16(h + off);
    }
    __device__ __forceinline__ float ld1(size_t off) const {
        return f ? f[off] : (float)h[off];
    }
};
inline YRef yref(const void* f32, const void* bf16) {
    return YRef{static_cast<const float*>(f32), f32 ? nullptr : static_cast<const __bf16*>(bf16)};
}
inline YRef yref(const ugpg_src_t& s) { return yref(s.data, s.data_bf16); }

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

// BatchNorm(+ReLU) backward of one element: g = da*[scale*y + shift > 0], xhat =
// (y - mean)*invstd, dy = (g - mean(g) - xhat*mean(g*xhat))*scale (k0 = mean(g), k1 =
// mean(g*xhat) from bn_bwd_finalize).  One definition with contraction off for every
// kernel that forms dy -- the BatchNorm-backward apply and the weight gradient that forms
// it while loading (WgradArgs.bn_*) -- so both give bit-identical dy.
__device__ __forceinline__ float bn_bwd_dy(float d, float v, float sc, float sh, float mu,
                                           float is, float k0, float k1) {
#pragma clang fp contract(off)
    const float g = fmaf(v, sc, sh) > 0.f ? d : 0.f;
    const float xh = (v - mu) * is;
    return fmaf(-xh, k1, g - k0) * sc;
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

// BatchNorm-backward partials folded into the kernel that produces da = dL/d(relu(bn(y)))
// (ugpg_bnb_t): g = da*[scale*y+shift > 0], xhat = (y-mean)*invstd, per block and
// channel sum g, sum g*xhat, sum xhat -> part[3][C][nblk] (the layout of bn.hip's
// bn_bwd_reduce_kernel, finalized by ugpg_bn_relu_bwd_partials).  Thread layout of that
// kernel: C/4 threads per pixel (4 channels each), 256/(C/4) pixel slots per block.
struct BnbArgs {
    YRef y;
    const float* mean;
    const float* invstd;
    const float* scale;
    const float* shift;
    float* part;
    int nblk;
    int64_t ppb;  // pixels per block
};
struct BnbAcc {
    f32x4 mu, is, sc, sh, sg, sgx, sx;
    __device__ void init(const BnbArgs& b, int c) {
        mu = *reinterpret_cast<const f32x4*>(b.mean + c);
        is = *reinterpret_cast<const f32x4*>(b.invstd + c);
        sc = *reinterpret_cast<const f32x4*>(b.scale + c);
        sh = *reinterpret_cast<const f32x4*>(b.shift + c);
        sg = sgx = sx = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __device__ void add(f32x4 d, f32x4 v) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float g = fmaf(v[k], sc[k], sh[k]) > 0.f ? d[k] : 0.f;
            const float xh = (v[k] - mu[k]) * is[k];
            sg[k] += g;
            sgx[k] = fmaf(g, xh, sgx[k]);
            sx[k] += xh;
        }
    }
    // block reduction over the pixel slots (fixed order) and the partial write; every
    // thread of the block calls it (LDS: 3 x 256 f32x4)
    __device__ void write(const BnbArgs& b, int C) {
        __shared__ f32x4 rs[256], rq[256], rx[256];
        const int tid = threadIdx.x, c4n = C / 4, slots = 256 / c4n;
        const int q = tid % c4n, slot = tid / c4n;
        rs[tid] = sg;
        rq[tid] = sgx;
        rx[tid] = sx;
        __syncthreads();
        if (slot == 0) {
            f32x4 a = sg, g2 = sgx, x = sx;
            for (int s2 = 1; s2 < slots; ++s2) {
                a += rs[s2 * c4n + q];
                g2 += rq[s2 * c4n + q];
                x += rx[s2 * c4n + q];
            }
            const int c = 4 * q;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                b.part[(size_t)(c + k) * b.nblk + blockIdx.x] = a[k];
                b.part[((size_t)C + c + k) * b.nblk + blockIdx.x] = g2[k];
                b.part[((size_t)2 * C + c + k) * b.nblk + blockIdx.x] = x[k];
            }
        }
    }
};

}  // namespace ugpg
