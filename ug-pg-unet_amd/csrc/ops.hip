// Memory-bound kernels of the UG-PG-UNet hot path (gfx950, fp32):
//   MaxPool2d(2)          UG_unet_parts.py:49                 (K8)
//   bilinear x2 / resize  UG_unet_parts.py:78, UG_unet.py:36-53 (K9, K12)
//   uncertainty map       UG_unet.py:45-57                      (K13)
//   1x1 heads + sum       UG_unet_parts.py:84-91, UG_unet.py:294-303 (K11)
//   weighted BCE          UG_unet.py:61-94, uncertainty_guided_trainer.py:64-65 (K13)
//   Dice / accuracy       uncertainty_guided_trainer.py:90-123 (K14)
//   RMSprop               uncertainty_guided_trainer.py:84-88  (K15)
//   avgpool/Linear head   Herlev/train_herlev.py:66-77         (K16)
// All reductions are deterministic (fixed-order block partials, fp64 merge).
#include <algorithm>

#include "common.h"

namespace ugpg {

// ---------------------------------------------------------------- max-pool
// (NT = nontemporal window loads: measured neutral, instantiated off)

template <bool NT>
__global__ void maxpool2_fwd_kernel(YRef x, const float* sc, const float* sh, int B, int H,
                                    int W, int C, float* out, __bf16* out16, uint8_t* am) {
    const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
    const int64_t total = (int64_t)B * Ho * Wo * C4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        int64_t r = i / C4;
        const int ox = (int)(r % Wo);
        r /= Wo;
        const int oy = (int)(r % Ho), b = (int)(r / Ho);
        f32x4 best;
        uint8_t idx[4] = {0, 0, 0, 0};
        f32x4 xv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int y = 2 * oy + (k >> 1), xx = 2 * ox + (k & 1);
            const size_t off = ((size_t)(b * H + y) * W + xx) * C + c;
            // NT: the window is read once here; the skip connection re-reads the block's
            // output only several layers later, long after it would have left the caches
            xv[k] = NT && x.f ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x.f + off))
                              : x.ld4(off);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f32x4 v = act_apply4(xv[k], sc, sh, c);
            if (k == 0) {
                best = v;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (v[j] > best[j] || isnan(v[j])) {
                        best[j] = v[j];
                        idx[j] = (uint8_t)k;
                    }
            }
        }
        if (out) {
            *reinterpret_cast<f32x4*>(out + i * 4) = best;
        } else {  // bf16 storage (RNE): the next conv's bf16 operand, exactly
            typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
            typedef float f32x2_t __attribute__((ext_vector_type(2)));
            const unsigned lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{best.x, best.y}, bf16x2_t));
            const unsigned hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{best.z, best.w}, bf16x2_t));
            *reinterpret_cast<uint2*>(out16 + i * 4) = uint2{lo, hi};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) am[i * 4 + j] = idx[j];
    }
}

// bf16 storage in and out (the bf16 arithmetic): 8 channels per thread, one 16-byte load per
// window pixel and one 16-byte store (the 4-channel form moved 8 bytes per access and ran at
// 2.4-3.5 TB/s).  Per element the same arithmetic, max rule and argmax as the fp32 form.
__device__ __forceinline__ void ld8_bf16(const __bf16* p, f32x4& lo, f32x4& hi) {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    lo = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
               __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
    hi = f32x4{__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
               __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
}
__device__ __forceinline__ unsigned pk2_bf16(float a, float b) {  // round to nearest even
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    typedef float f32x2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}
__device__ __forceinline__ void st8_bf16(__bf16* p, const f32x4& lo, const f32x4& hi) {
    *reinterpret_cast<uint4*>(p) =
        uint4{pk2_bf16(lo.x, lo.y), pk2_bf16(lo.z, lo.w), pk2_bf16(hi.x, hi.y), pk2_bf16(hi.z, hi.w)};
}

__device__ __forceinline__ f32x4 act4c(f32x4 v, const f32x4& s, const f32x4& h, bool on) {
    if (on) {
        v.x = fmaxf(fmaf(v.x, s.x, h.x), 0.0f);
        v.y = fmaxf(fmaf(v.y, s.y, h.y), 0.0f);
        v.z = fmaxf(fmaf(v.z, s.z, h.z), 0.0f);
        v.w = fmaxf(fmaf(v.w, s.w, h.w), 0.0f);
    }
    return v;
}

// A thread keeps its 8 channels (the grid stride, a multiple of 256, is a multiple of C/8),
// so the activation coefficients are loaded once; U units' window loads go out before the
// first is used.
__global__ void __launch_bounds__(256) maxpool2_fwd16_kernel(const __bf16* x, const float* sc,
                                                             const float* sh, int B, int H, int W,
                                                             int C, __bf16* out16, uint8_t* am) {
    constexpr int U = 4;
    const int Ho = H / 2, Wo = W / 2, C8 = C / 8;
    const int64_t total = (int64_t)B * Ho * Wo * C8, G = (int64_t)gridDim.x * blockDim.x;
    int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i0 >= total) return;
    const int c = (int)(i0 % C8) * 8;
    const bool on = sc != nullptr;
    f32x4 s4[2], h4[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        s4[hf] = on ? *reinterpret_cast<const f32x4*>(sc + c + 4 * hf) : f32x4{1.f, 1.f, 1.f, 1.f};
        h4[hf] = on ? *reinterpret_cast<const f32x4*>(sh + c + 4 * hf) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (; i0 < total; i0 += U * G) {
        f32x4 xv[U][4][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = min(i0 + u * G, total - 1);
            // 32-bit index arithmetic (the host launches this form for < 2^32 units): four
            // 64-bit divisions per unit held the kernel at 3.7 TB/s
            uint32_t r = (uint32_t)i / (uint32_t)C8;
            const int ox = (int)(r % (uint32_t)Wo);
            r /= (uint32_t)Wo;
            const int oy = (int)(r % (uint32_t)Ho), b = (int)(r / (uint32_t)Ho);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int y = 2 * oy + (k >> 1), xx = 2 * ox + (k & 1);
                ld8_bf16(x + ((size_t)(b * H + y) * W + xx) * C + c, xv[u][k][0], xv[u][k][1]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * G;
            if (i >= total) break;
            f32x4 best[2];
            uint8_t idx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const f32x4 v = act4c(xv[u][k][hf], s4[hf], h4[hf], on);
                    if (k == 0) {
                        best[hf] = v;
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (v[j] > best[hf][j] || isnan(v[j])) {
                                best[hf][j] = v[j];
                                idx[4 * hf + j] = (uint8_t)k;
                            }
                    }
                }
            st8_bf16(out16 + i * 8, best[0], best[1]);
            unsigned lo = 0, hi = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lo |= (unsigned)idx[j] << (8 * j);
                hi |= (unsigned)idx[4 + j] << (8 * j);
            }
            *reinterpret_cast<uint2*>(am + i * 8) = uint2{lo, hi};
        }
    }
}

__global__ void maxpool2_bwd_kernel(const float* dout, const uint8_t* am, int B, int H, int W,
                                    int C, float* din, int acc) {
    const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
    const int64_t total = (int64_t)B * H * W * C4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        int64_t r = i / C4;
        const int x = (int)(r % W);
        r /= W;
        const int y = (int)(r % H), b = (int)(r / H);
        f32x4 g = {0.f, 0.f, 0.f, 0.f};
        const int oy = y >> 1, ox = x >> 1;
        if (oy < Ho && ox < Wo) {
            const int k = (y & 1) * 2 + (x & 1);
            const size_t o = ((size_t)(b * Ho + oy) * Wo + ox) * C + c;
            const f32x4 d = *reinterpret_cast<const f32x4*>(dout + o);
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = am[o + j] == k ? d[j] : 0.f;
        }
        f32x4* dst = reinterpret_cast<f32x4*>(din + i * 4);
        if (acc) g += *dst;
        *dst = g;
    }
}

// maxpool backward fused with the BatchNorm-backward partials of its output (the BN of
// the block whose activation was pooled: this gather is the last writer of its da).
// Block = a contiguous pixel range, thread = 4 channels of every slots-th pixel.
// STORE false: the partials only (din is read when acc, never written) -- the routed
// gradient is recomputed by the BatchNorm-backward apply (ugpg_bn_relu_bwd_partials_routed)
template <bool STORE>
__global__ void __launch_bounds__(256)
    maxpool2_bwd_bnb_kernel(const float* dout, const uint8_t* am, int B, int H, int W, int C,
                            float* din, int acc, BnbArgs bnb) {
    // U pixels' loads go out before the first is used, with 32-bit pixel coordinates (the
    // host requires B*H*W < 2^31): the four 64-bit divisions per pixel and one pixel's loads
    // in flight per thread held the pass at 4.75-5.07 TB/s.  Same sums in the same order.
    constexpr int U = 4;
    const int Ho = H / 2, Wo = W / 2, c4n = C / 4, slots = 256 / c4n;
    const int tid = threadIdx.x, q = tid % c4n, slot = tid / c4n, c = 4 * q;
    const int64_t npix = (int64_t)B * H * W;
    BnbAcc st;
    st.init(bnb, c);
    if (slot < slots) {
        const int64_t p0 = blockIdx.x * bnb.ppb, p1 = min(npix, p0 + bnb.ppb);
        for (int64_t p = p0 + slot; p < p1; p += U * slots) {
            f32x4 d[U], base[U], yv[U];
            uchar4 m[U];
            int k[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t pc = (uint32_t)min(p + u * slots, p1 - 1);  // (clamped: loads only)
                const uint32_t x = pc % (uint32_t)W, r = pc / (uint32_t)W;
                const uint32_t yy = r % (uint32_t)H, b = r / (uint32_t)H;
                const uint32_t oy = yy >> 1, ox = x >> 1;
                const bool in = oy < (uint32_t)Ho && ox < (uint32_t)Wo;
                k[u] = in ? (int)((yy & 1) * 2 + (x & 1)) : -1;  // -1: outside the pooled area
                const size_t o = in ? ((size_t)(b * Ho + oy) * Wo + ox) * C + c : (size_t)c;
                d[u] = *reinterpret_cast<const f32x4*>(dout + o);
                m[u] = *reinterpret_cast<const uchar4*>(am + o);
                base[u] = acc ? *reinterpret_cast<const f32x4*>(din + (size_t)pc * C + c)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
                yv[u] = bnb.y.ld4((size_t)pc * C + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t pu = p + u * slots;
                if (pu >= p1) break;
                f32x4 g;
                g[0] = m[u].x == k[u] ? d[u][0] : 0.f;
                g[1] = m[u].y == k[u] ? d[u][1] : 0.f;
                g[2] = m[u].z == k[u] ? d[u][2] : 0.f;
                g[3] = m[u].w == k[u] ? d[u][3] : 0.f;
                if (acc) g += base[u];
                if constexpr (STORE) *reinterpret_cast<f32x4*>(din + pu * C + c) = g;
                st.add(g, yv[u]);
            }
        }
    }
    st.write(bnb, C);
}

// fp32 <-> bf16 casts of a gradient bucket (the bf16 gradient exchange of config 3):
// round to nearest even, NaN kept quiet
__global__ void cast_f32_bf16_kernel(const float* in, uint16_t* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t u = __float_as_uint(in[i]);
        out[i] = (u & 0x7fffffffu) > 0x7f800000u
                     ? (uint16_t)((u >> 16) | 0x40u)
                     : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
}
__global__ void cast_bf16_f32_kernel(const uint16_t* in, float* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = __uint_as_float((uint32_t)in[i] << 16);
}

// ------------------------------------------------- bilinear (align_corners)
// gather-form backward: input index i collects from outputs o with i0(o)==i or i1(o)==i
__device__ __forceinline__ void ac_range(int i, int in, int out, int& lo, int& hi) {
    if (in == out) {
        lo = hi = i;
        return;
    }
    if (out == 1) {
        lo = 0;
        hi = 0;
        return;
    }
    const float scale = (float)(in - 1) / (float)(out - 1);
    if (scale <= 0.f) {
        lo = 0;
        hi = out - 1;
        return;
    }
    lo = (int)floorf((float)(i - 1) / scale) - 1;
    hi = (int)ceilf((float)(i + 1) / scale) + 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > out - 1 ? out - 1 : hi;
}

__device__ __forceinline__ float ac_weight(int o, int i, int in, int out) {
    int i0, i1;
    float l0, l1;
    ac_index(o, in, out, i0, i1, l0, l1);
    float w = 0.f;
    if (i0 == i) w += l0;
    if (i1 == i) w += l1;
    return w;
}

// ac_range is conservative (about 2/scale + 5 candidates, most of zero weight: 7 per
// dimension for x2, 49 ac_weight evaluations per input quad); trimming the zero-weight
// ends leaves the 2-3 real contributors.  The skipped terms had zero weight and were
// skipped anyway, so sums and their order are unchanged.
__device__ __forceinline__ void ac_range_tight(int i, int in, int out, int& lo, int& hi) {
    ac_range(i, in, out, lo, hi);
    while (lo < hi && ac_weight(lo, i, in, out) == 0.f) ++lo;
    while (hi > lo && ac_weight(hi, i, in, out) == 0.f) --hi;
}

// Row-blocked forms: blockIdx.y = output (input) row, so the row's interpolation
// indices/weights and the 64-bit image offsets are computed once per thread, and a
// thread keeps one channel quad (the x-stride is a multiple of C/4), loading the lazy
// BatchNorm coefficients once.  Same arithmetic, same order as the flat forms.
__global__ void bilinear_nhwc_fwd_kernel(YRef x, const float* sc, const float* sh, int B,
                                         int Hi, int Wi, int C, float* out, __bf16* out16,
                                         int Ho, int Wo) {
    const int C4 = C / 4;
    const int row = blockIdx.y;  // b * Ho + oy
    const int b = row / Ho, oy = row % Ho;
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    ac_index(oy, Hi, Ho, y0, y1, ly0, ly1);
    const size_t r0 = ((size_t)b * Hi + y0) * Wi * C;  // element offsets of the two rows
    const size_t r1 = ((size_t)b * Hi + y1) * Wi * C;
    const size_t orow = (size_t)row * Wo * C;
    // out16 (out == nullptr): bf16 storage of the result (the bf16 arithmetic's conv input)
    auto store = [&](size_t e, f32x4 v) {
        if (out16) {
            typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf4*>(out16 + e) = bf4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        } else {
            *reinterpret_cast<f32x4*>(out + e) = v;
        }
    };
    const int n = Wo * C4, stride = gridDim.x * blockDim.x;
    const bool fixed_c = stride % C4 == 0;  // then a thread keeps its channel quad
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int c = (t % C4) * 4;
    f32x4 s4 = {1.f, 1.f, 1.f, 1.f}, h4 = {0.f, 0.f, 0.f, 0.f};
    auto coef = [&]() {
        if (sc) {
            s4 = *reinterpret_cast<const f32x4*>(sc + c);
            h4 = *reinterpret_cast<const f32x4*>(sh + c);
        }
    };
    coef();
    auto act = [&](f32x4 v) {
        if (sc) {
            v.x = fmaxf(fmaf(v.x, s4.x, h4.x), 0.0f);
            v.y = fmaxf(fmaf(v.y, s4.y, h4.y), 0.0f);
            v.z = fmaxf(fmaf(v.z, s4.z, h4.z), 0.0f);
            v.w = fmaxf(fmaf(v.w, s4.w, h4.w), 0.0f);
        }
        return v;
    };
    constexpr int U = 4;
    if (fixed_c && n % (U * stride) == 0) {
        // U output quads per thread, all 4U loads issued before the first store
        // (uniform trip count: no predication, the operands stay in VGPRs)
        const int step = stride / C4;  // output pixels between a thread's quads
        for (; t < n; t += U * stride) {
            const int ox0 = t / C4;
            f32x4 a[U][4];
            float wx0[U], wx1[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                ac_index(ox0 + u * step, Wi, Wo, x0, x1, wx0[u], wx1[u]);
                a[u][0] = x.ld4(r0 + (size_t)x0 * C + c);
                a[u][1] = x.ld4(r0 + (size_t)x1 * C + c);
                a[u][2] = x.ld4(r1 + (size_t)x0 * C + c);
                a[u][3] = x.ld4(r1 + (size_t)x1 * C + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const f32x4 a00 = act(a[u][0]), a01 = act(a[u][1]), a10 = act(a[u][2]),
                            a11 = act(a[u][3]);
                const f32x4 v = ly0 * (wx0[u] * a00 + wx1[u] * a01) +
                                ly1 * (wx0[u] * a10 + wx1[u] * a11);
                store(orow + (size_t)(ox0 + u * step) * C + c, v);
            }
        }
        return;
    }
    for (; t < n; t += stride) {
        if (!fixed_c) {
            c = (t % C4) * 4;
            coef();
        }
        const int ox = t / C4;
        ac_index(ox, Wi, Wo, x0, x1, lx0, lx1);
        const f32x4 a00 = act(x.ld4(r0 + (size_t)x0 * C + c));
        const f32x4 a01 = act(x.ld4(r0 + (size_t)x1 * C + c));
        const f32x4 a10 = act(x.ld4(r1 + (size_t)x0 * C + c));
        const f32x4 a11 = act(x.ld4(r1 + (size_t)x1 * C + c));
        const f32x4 v = ly0 * (lx0 * a00 + lx1 * a01) + ly1 * (lx0 * a10 + lx1 * a11);
        store(orow + (size_t)ox * C + c, v);
    }
}

// bf16 in and out, 8 channels per thread (see maxpool2_fwd16_kernel), one block per output
// row, U units' loads issued before the first is used; per element the same arithmetic and
// order as bilinear_nhwc_fwd_kernel.
__global__ void __launch_bounds__(256) bilinear_nhwc_fwd16_kernel(const __bf16* x, const float* sc,
                                                                  const float* sh, int B, int Hi,
                                                                  int Wi, int C, __bf16* out16,
                                                                  int Ho, int Wo) {
    constexpr int U = 4;
    const int C8 = C / 8;
    const int row = blockIdx.y;  // b * Ho + oy
    const int b = row / Ho, oy = row % Ho;
    int y0, y1;
    float ly0, ly1;
    ac_index(oy, Hi, Ho, y0, y1, ly0, ly1);
    const size_t r0 = ((size_t)b * Hi + y0) * Wi * C, r1 = ((size_t)b * Hi + y1) * Wi * C;
    const size_t orow = (size_t)row * Wo * C;
    const int n = Wo * C8, G = gridDim.x * blockDim.x;
    int t0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 >= n) return;
    const int c = (t0 % C8) * 8;  // fixed: G is a multiple of 256, hence of C8
    const bool on = sc != nullptr;
    f32x4 s4[2], h4[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        s4[hf] = on ? *reinterpret_cast<const f32x4*>(sc + c + 4 * hf) : f32x4{1.f, 1.f, 1.f, 1.f};
        h4[hf] = on ? *reinterpret_cast<const f32x4*>(sh + c + 4 * hf) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (; t0 < n; t0 += U * G) {
        f32x4 a[U][4][2];
        float wx0[U], wx1[U];
        int oxs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = min(t0 + u * G, n - 1);
            const int ox = t / C8;
            int x0, x1;
            ac_index(ox, Wi, Wo, x0, x1, wx0[u], wx1[u]);
            oxs[u] = ox;
            ld8_bf16(x + r0 + (size_t)x0 * C + c, a[u][0][0], a[u][0][1]);
            ld8_bf16(x + r0 + (size_t)x1 * C + c, a[u][1][0], a[u][1][1]);
            ld8_bf16(x + r1 + (size_t)x0 * C + c, a[u][2][0], a[u][2][1]);
            ld8_bf16(x + r1 + (size_t)x1 * C + c, a[u][3][0], a[u][3][1]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t0 + u * G >= n) break;
            f32x4 v[2];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const f32x4 a00 = act4c(a[u][0][hf], s4[hf], h4[hf], on),
                            a01 = act4c(a[u][1][hf], s4[hf], h4[hf], on),
                            a10 = act4c(a[u][2][hf], s4[hf], h4[hf], on),
                            a11 = act4c(a[u][3][hf], s4[hf], h4[hf], on);
                v[hf] = ly0 * (wx0[u] * a00 + wx1[u] * a01) + ly1 * (wx0[u] * a10 + wx1[u] * a11);
            }
            st8_bf16(out16 + orow + (size_t)oxs[u] * C + c, v[0], v[1]);
        }
    }
}

__global__ void bilinear_nhwc_bwd_kernel(const float* dout, int B, int Ho, int Wo, int C,
                                         float* din, int Hi, int Wi, int acc) {
    const int C4 = C / 4;
    const int row = blockIdx.y;  // b * Hi + iy
    const int b = row / Hi, iy = row % Hi;
    int ylo, yhi;
    ac_range_tight(iy, Hi, Ho, ylo, yhi);
    const int n = Wi * C4, stride = gridDim.x * blockDim.x;
    // x2-type ranges (<= 4 contributors per dimension): weights hoisted, all loads
    // issued before the first accumulate, same terms in the same order as the loop form
    float wy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wy[j] = ylo + j <= yhi ? ac_weight(ylo + j, iy, Hi, Ho) : 0.f;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
        const int c = (t % C4) * 4, ix = t / C4;
        int xlo, xhi;
        ac_range_tight(ix, Wi, Wo, xlo, xhi);
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        if (yhi - ylo <= 3 && xhi - xlo <= 3) {
            float wx[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) wx[k] = xlo + k <= xhi ? ac_weight(xlo + k, ix, Wi, Wo) : 0.f;
            f32x4 d[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    d[j][k] = wy[j] != 0.f && wx[k] != 0.f
                                  ? *reinterpret_cast<const f32x4*>(
                                        dout + ((size_t)(b * Ho + ylo + j) * Wo + xlo + k) * C + c)
                                  : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (wy[j] != 0.f && wx[k] != 0.f) s += (wy[j] * wx[k]) * d[j][k];
            f32x4* dst = reinterpret_cast<f32x4*>(din + ((size_t)row * Wi + ix) * C + c);
            if (acc) s += *dst;
            *dst = s;
            continue;
        }
        for (int oy = ylo; oy <= yhi; ++oy) {
            const float wyk = ac_weight(oy, iy, Hi, Ho);
            if (wyk == 0.f) continue;
            for (int ox = xlo; ox <= xhi; ++ox) {
                const float wx = ac_weight(ox, ix, Wi, Wo);
                if (wx == 0.f) continue;
                const f32x4 d = *reinterpret_cast<const f32x4*>(
                    dout + ((size_t)(b * Ho + oy) * Wo + ox) * C + c);
                s += (wyk * wx) * d;
            }
        }
        f32x4* dst = reinterpret_cast<f32x4*>(din + ((size_t)row * Wi + ix) * C + c);
        if (acc) s += *dst;
        *dst = s;
    }
}

// bilinear backward fused with the BatchNorm-backward partials of din (the BN of the
// block whose activation was upsampled: this gather is the last writer of its da).
// The body of bilinear_nhwc_bwd_kernel (bit-identical din) with one workgroup per input
// row (its partial slot: nslots = B * Hi), whose threads keep one 4-channel group each
// (256 % (C/4) == 0).
__global__ void __launch_bounds__(256)
    bilinear_nhwc_bwd_bnb_kernel(const float* dout, int B, int Ho, int Wo, int C, float* din,
                                 int Hi, int Wi, int acc, BnbArgs bnb) {
    const int C4 = C / 4;
    const int row = blockIdx.x;  // b * Hi + iy
    const int b = row / Hi, iy = row % Hi;
    BnbAcc st;
    st.init(bnb, (threadIdx.x % C4) * 4);
    int ylo, yhi;
    ac_range_tight(iy, Hi, Ho, ylo, yhi);
    const int n = Wi * C4;
    float wy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wy[j] = ylo + j <= yhi ? ac_weight(ylo + j, iy, Hi, Ho) : 0.f;
    // the column ranges and weights of the row's input columns, once per workgroup (C/4
    // threads shared each column's, and evaluated it per element: ac_range_tight's loops and
    // ac_weight's index arithmetic made this pass VALU-bound); the same values, so the same sums
    constexpr int TAB = 256;
    __shared__ int txlo[TAB], txhi[TAB];
    __shared__ float twx[4][TAB];
    const bool tab = Wi <= TAB;  // (uniform)
    if (tab) {
        for (int ix = threadIdx.x; ix < Wi; ix += blockDim.x) {
            int xlo, xhi;
            ac_range_tight(ix, Wi, Wo, xlo, xhi);
            txlo[ix] = xlo;
            txhi[ix] = xhi;
#pragma unroll
            for (int k = 0; k < 4; ++k) twx[k][ix] = xlo + k <= xhi ? ac_weight(xlo + k, ix, Wi, Wo) : 0.f;
        }
        __syncthreads();
    }
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        const int c = (t % C4) * 4, ix = t / C4;
        int xlo, xhi;
        if (tab) {
            xlo = txlo[ix];
            xhi = txhi[ix];
        } else {
            ac_range_tight(ix, Wi, Wo, xlo, xhi);
        }
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        if (yhi - ylo <= 3 && xhi - xlo <= 3) {
            float wx[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                wx[k] = tab ? twx[k][ix] : xlo + k <= xhi ? ac_weight(xlo + k, ix, Wi, Wo) : 0.f;
            f32x4 d[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    d[j][k] = wy[j] != 0.f && wx[k] != 0.f
                                  ? *reinterpret_cast<const f32x4*>(
                                        dout + ((size_t)(b * Ho + ylo + j) * Wo + xlo + k) * C + c)
                                  : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (wy[j] != 0.f && wx[k] != 0.f) s += (wy[j] * wx[k]) * d[j][k];
        } else {
            for (int oy = ylo; oy <= yhi; ++oy) {
                const float wyk = ac_weight(oy, iy, Hi, Ho);
                if (wyk == 0.f) continue;
                for (int ox = xlo; ox <= xhi; ++ox) {
                    const float wx = ac_weight(ox, ix, Wi, Wo);
                    if (wx == 0.f) continue;
                    const f32x4 d = *reinterpret_cast<const f32x4*>(
                        dout + ((size_t)(b * Ho + oy) * Wo + ox) * C + c);
                    s += (wyk * wx) * d;
                }
            }
        }
        const size_t o = ((size_t)row * Wi + ix) * C + c;
        f32x4* dst = reinterpret_cast<f32x4*>(din + o);
        if (acc) s += *dst;
        *dst = s;
        st.add(s, bnb.y.ld4(o));
    }
    st.write(bnb, C);
}

// ------------------------------------------------------------- NCHW resize
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ int nearest_src(int o, int in, int out) {
    if (in == out) return o;
    if (out == 2 * in) return o >> 1;
    const float scale = (float)in / (float)out;
    const int s = (int)floorf((float)o * scale);
    return s < in - 1 ? s : in - 1;
}

__global__ void resize_nchw_kernel(const float* in, int BC, int Hi, int Wi, float* out, int Ho,
                                   int Wo, int mode) {
    const int64_t total = (int64_t)BC * Ho * Wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int ox = (int)(i % Wo);
        int64_t r = i / Wo;
        const int oy = (int)(r % Ho);
        const int64_t bc = r / Ho;
        const float* src = in + bc * Hi * Wi;
        float v;
        if (mode == 1) {
            v = src[(size_t)nearest_src(oy, Hi, Ho) * Wi + nearest_src(ox, Wi, Wo)];
        } else {
            int y0, y1, x0, x1;
            float ly0, ly1, lx0, lx1;
            ac_index(oy, Hi, Ho, y0, y1, ly0, ly1);
            ac_index(ox, Wi, Wo, x0, x1, lx0, lx1);
            float a00 = src[(size_t)y0 * Wi + x0], a01 = src[(size_t)y0 * Wi + x1];
            float a10 = src[(size_t)y1 * Wi + x0], a11 = src[(size_t)y1 * Wi + x1];
            if (mode == 2) {
                a00 = sigmoidf_(a00);
                a01 = sigmoidf_(a01);
                a10 = sigmoidf_(a10);
                a11 = sigmoidf_(a11);
            }
            v = ly0 * (lx0 * a00 + lx1 * a01) + ly1 * (lx0 * a10 + lx1 * a11);
            if (mode == 2) v = 1.0f - 2.0f * fabsf(v - 0.5f);
        }
        out[i] = v;
    }
}

// gradient of resize_nchw mode 0 (bilinear, align_corners=True; ProgressiveUNet.forward's
// input resize, UG_unet.py:418-424): gather form -- each input pixel sums w_y * w_x * dy
// over the outputs whose interpolation reads it (the same index/weight arithmetic as the
// forward), deterministic, no atomics.
__global__ void resize_nchw_bwd_kernel(const float* dout, int BC, int Ho, int Wo, float* din,
                                       int Hi, int Wi) {
    const int64_t total = (int64_t)BC * Hi * Wi;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % Wi);
        const int64_t r = i / Wi;
        const int y = (int)(r % Hi);
        const int64_t bc = r / Hi;
        const float* g = dout + bc * Ho * Wo;
        int ylo, yhi, xlo, xhi;
        ac_range_tight(y, Hi, Ho, ylo, yhi);
        ac_range_tight(x, Wi, Wo, xlo, xhi);
        float acc = 0.f;
        for (int oy = ylo; oy <= yhi; ++oy) {
            const float wy = ac_weight(oy, y, Hi, Ho);
            if (wy == 0.f) continue;
            float row = 0.f;
            for (int ox = xlo; ox <= xhi; ++ox) {
                const float wx = ac_weight(ox, x, Wi, Wo);
                if (wx != 0.f) row = fmaf(wx, g[(size_t)oy * Wo + ox], row);
            }
            acc = fmaf(wy, row, acc);
        }
        din[i] = acc;
    }
}

// One pixel per thread: C coalesced plane reads and, for Cp % 4 == 0, Cp/4 16-byte stores;
// one division per pixel (the element-per-thread form's three 64-bit divisions per value
// ran at 1.7 TB/s)
template <bool V4>
__global__ void nchw_to_nhwc_kernel(const float* in, int B, int C, int HW, float* out, int Cp) {
    const int64_t npix = (int64_t)B * HW;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < npix;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = q / HW, p = q - b * HW;
        const float* src = in + (size_t)b * C * HW + p;
        float* dst = out + (size_t)q * Cp;
        if constexpr (V4) {
            for (int c4 = 0; c4 < Cp; c4 += 4) {
                f32x4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = c4 + i < C ? src[(size_t)(c4 + i) * HW] : 0.f;
                *reinterpret_cast<f32x4*>(dst + c4) = v;
            }
        } else {
            for (int c = 0; c < Cp; ++c) dst[c] = c < C ? src[(size_t)c * HW] : 0.f;
        }
    }
}

__global__ void nhwc_to_nchw_kernel(const float* in, int B, int C, int HW, int Cs, float* out,
                                    int acc) {
    const int64_t total = (int64_t)B * C * HW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i % HW);
        const int64_t r = i / HW;
        const int c = (int)(r % C), b = (int)(r / C);
        const float v = in[((size_t)b * HW + p) * Cs + c];
        out[i] = acc ? out[i] + v : v;
    }
}

// ------------------------------------------------------------------ heads
// 16 lanes per pixel; lane16 owns channels {4*l16 + 64*j}.
constexpr int HEAD_NC_MAX = 4, HEAD_CJ_MAX = 4;

__global__ void __launch_bounds__(256) head_fwd_kernel(YRef x, const float* sc,
                                                       const float* sh, int64_t npix, int C,
                                                       const float* w, const float* bias, int nc,
                                                       float* h) {
    const int l16 = threadIdx.x & 15, CJ = C / 64;
    for (int64_t p = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 4; p < npix;
         p += ((int64_t)gridDim.x * blockDim.x) >> 4) {
        float acc[HEAD_NC_MAX] = {0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < CJ; ++j) {
            const int c = l16 * 4 + 64 * j;
            const f32x4 v = act_apply4(x.ld4(p * C + c), sc, sh, c);
            for (int k = 0; k < nc; ++k) {
                const f32x4 wv = *reinterpret_cast<const f32x4*>(w + (size_t)k * C + c);
                acc[k] += v.x * wv.x + v.y * wv.y + v.z * wv.z + v.w * wv.w;
            }
        }
        for (int k = 0; k < nc; ++k) {
            float s = acc[k];
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
            if (l16 == 0) h[p * nc + k] = s + bias[k];
        }
    }
}

// The same head with the C/64 channel groups a compile-time count: the lane's activation
// coefficients and head weights are loaded once per thread (not per pixel), and four
// pixels' loads go out before the first is used (the per-pixel form ran at 3.3 TB/s).
// Arithmetic and reduction order are those of head_fwd_kernel (bit-identical).
template <int CJ>
__global__ void __launch_bounds__(256) head_fwd_cj_kernel(YRef x, const float* sc,
                                                          const float* sh, int64_t npix,
                                                          const float* w, const float* bias,
                                                          int nc, float* h) {
    constexpr int C = 64 * CJ, U = 4;
    const int l16 = threadIdx.x & 15;
    f32x4 ws[CJ][HEAD_NC_MAX], as[CJ], ah[CJ];
#pragma unroll
    for (int j = 0; j < CJ; ++j) {
        const int c = l16 * 4 + 64 * j;
        as[j] = sc ? *reinterpret_cast<const f32x4*>(sc + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        ah[j] = sc ? *reinterpret_cast<const f32x4*>(sh + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < HEAD_NC_MAX; ++k)
            ws[j][k] = k < nc ? *reinterpret_cast<const f32x4*>(w + (size_t)k * C + c)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int64_t G = ((int64_t)gridDim.x * blockDim.x) >> 4;
    for (int64_t p0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 4; p0 < npix;
         p0 += U * G) {
        f32x4 v[U][CJ];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t p = min(p0 + u * G, npix - 1);
#pragma unroll
            for (int j = 0; j < CJ; ++j)
                v[u][j] = x.ld4(p * C + l16 * 4 + 64 * j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t p = p0 + u * G;
            float acc[HEAD_NC_MAX] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                f32x4 a = v[u][j];
                if (sc) {
                    a.x = fmaxf(fmaf(a.x, as[j].x, ah[j].x), 0.0f);
                    a.y = fmaxf(fmaf(a.y, as[j].y, ah[j].y), 0.0f);
                    a.z = fmaxf(fmaf(a.z, as[j].z, ah[j].z), 0.0f);
                    a.w = fmaxf(fmaf(a.w, as[j].w, ah[j].w), 0.0f);
                }
#pragma unroll
                for (int k = 0; k < HEAD_NC_MAX; ++k)
                    if (k < nc)
                        acc[k] += a.x * ws[j][k].x + a.y * ws[j][k].y + a.z * ws[j][k].z +
                                  a.w * ws[j][k].w;
            }
#pragma unroll
            for (int k = 0; k < HEAD_NC_MAX; ++k) {
                if (k >= nc) break;
                float s = acc[k];
#pragma unroll
                for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
                if (l16 == 0 && p < npix) h[p * nc + k] = s + bias[k];
            }
        }
    }
}

// C = 64: 8 lanes per pixel, 8 channels per lane -- one 16-byte load per lane for a bf16 y
// (two for fp32), 8 products summed per lane and a 3-step butterfly: half the instructions
// per pixel of the 16-lane form, whose bf16 launch at 256^2 ran at 2.5 TB/s (the fp32 one
// at 4.7).  The same arithmetic for either storage (bit-identical when y is bf16-exact).
__global__ void __launch_bounds__(256) head_fwd8_kernel(YRef x, const float* sc, const float* sh,
                                                        int64_t npix, const float* w,
                                                        const float* bias, int nc, float* h) {
    constexpr int C = 64, U = 4;
    const int l8 = threadIdx.x & 7, c = 8 * l8;
    f32x4 ws[HEAD_NC_MAX][2], as[2], ah[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        as[hf] = sc ? *reinterpret_cast<const f32x4*>(sc + c + 4 * hf) : f32x4{0.f, 0.f, 0.f, 0.f};
        ah[hf] = sc ? *reinterpret_cast<const f32x4*>(sh + c + 4 * hf) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < HEAD_NC_MAX; ++k)
            ws[k][hf] = k < nc ? *reinterpret_cast<const f32x4*>(w + (size_t)k * C + c + 4 * hf)
                               : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int64_t G = ((int64_t)gridDim.x * blockDim.x) >> 3;
    for (int64_t p0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3; p0 < npix;
         p0 += U * G) {
        f32x4 v[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t o = (size_t)min(p0 + u * G, npix - 1) * C + c;
            if (x.f) {
                v[u][0] = *reinterpret_cast<const f32x4*>(x.f + o);
                v[u][1] = *reinterpret_cast<const f32x4*>(x.f + o + 4);
            } else {
                ld8_bf16(x.h + o, v[u][0], v[u][1]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t p = p0 + u * G;
            float acc[HEAD_NC_MAX] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                f32x4 a = v[u][hf];
                if (sc) {
                    a.x = fmaxf(fmaf(a.x, as[hf].x, ah[hf].x), 0.0f);
                    a.y = fmaxf(fmaf(a.y, as[hf].y, ah[hf].y), 0.0f);
                    a.z = fmaxf(fmaf(a.z, as[hf].z, ah[hf].z), 0.0f);
                    a.w = fmaxf(fmaf(a.w, as[hf].w, ah[hf].w), 0.0f);
                }
#pragma unroll
                for (int k = 0; k < HEAD_NC_MAX; ++k)
                    if (k < nc)
                        acc[k] += a.x * ws[k][hf].x + a.y * ws[k][hf].y + a.z * ws[k][hf].z +
                                  a.w * ws[k][hf].w;
            }
#pragma unroll
            for (int k = 0; k < HEAD_NC_MAX; ++k) {
                if (k >= nc) break;
                float s = acc[k];
#pragma unroll
                for (int o = 4; o > 0; o >>= 1) s += __shfl_xor(s, o, 8);
                if (l8 == 0 && p < npix) h[p * nc + k] = s + bias[k];
            }
        }
    }
}

struct HeadSet {
    const float* h[4];
    int res[4];
    int n;
};

// Four consecutive outputs of one row per thread (one 16-byte store), the row's vertical
// indices / weights computed once per head, 32-bit offsets within a head; the same
// arithmetic and head order as before (per output: ly0*(lx0*a + lx1*b) + ly1*(...), summed
// over heads in order), so the logits are bit-identical to the one-output-per-thread form.
__global__ void __launch_bounds__(256) heads_combine_kernel(HeadSet hs, int B, int H, int W, int nc,
                                                            float* logits) {
    const int W4 = W >> 2;
    const int64_t total4 = (int64_t)B * nc * H * W4;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < total4;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int x0o = (int)(q % W4) * 4;
        const int64_t r = q / W4;  // (b, k, y) row
        const int y = (int)(r % H);
        const int k = (int)((r / H) % nc), b = (int)(r / ((int64_t)H * nc));
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        // constant head indices: every kernel argument is read once, at the kernel start
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j >= hs.n) break;
            const int R = hs.res[j];
            const float* hp = hs.h[j] + (size_t)b * R * R * nc + k;
            f32x4 v;
            if (R == H) {
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = hp[(y * W + x0o + u) * nc];
            } else {
                int y0, y1;
                float ly0, ly1;
                ac_index(y, R, H, y0, y1, ly0, ly1);
                const float* r0 = hp + y0 * R * nc;
                const float* r1 = hp + y1 * R * nc;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    int x0, x1;
                    float lx0, lx1;
                    ac_index(x0o + u, R, W, x0, x1, lx0, lx1);
                    v[u] = ly0 * (lx0 * r0[x0 * nc] + lx1 * r0[x1 * nc]) +
                           ly1 * (lx0 * r1[x0 * nc] + lx1 * r1[x1 * nc]);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] = (j == 0) ? v[u] : s[u] + v[u];
        }
        *reinterpret_cast<f32x4*>(logits + r * W + x0o) = s;
    }
}

// One output per thread: widths that are not a multiple of 4 (any even width reaches here
// through PGUNet1's single max-pool, as in the reference).  Same arithmetic and order.
__global__ void heads_combine1_kernel(HeadSet hs, int B, int H, int W, int nc, float* logits) {
    const int64_t total = (int64_t)B * nc * H * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % W);
        int64_t r = i / W;
        const int y = (int)(r % H);
        r /= H;
        const int k = (int)(r % nc), b = (int)(r / nc);
        float s = 0.f;
        for (int j = 0; j < hs.n; ++j) {
            const int R = hs.res[j];
            const float* hp = hs.h[j] + (size_t)b * R * R * nc + k;
            float v;
            if (R == H) {
                v = hp[((size_t)y * W + x) * nc];
            } else {
                int y0, y1, x0, x1;
                float ly0, ly1, lx0, lx1;
                ac_index(y, R, H, y0, y1, ly0, ly1);
                ac_index(x, R, W, x0, x1, lx0, lx1);
                v = ly0 * (lx0 * hp[((size_t)y0 * R + x0) * nc] + lx1 * hp[((size_t)y0 * R + x1) * nc]) +
                    ly1 * (lx0 * hp[((size_t)y1 * R + x0) * nc] + lx1 * hp[((size_t)y1 * R + x1) * nc]);
            }
            s = (j == 0) ? v : s + v;
        }
        logits[i] = s;
    }
}

// dh (NHWC, R x R, nc) from NCHW dlogits (H x W): the transpose of the align-corners
// upsample R -> H.  One block per (b, iy); for R < 256 the threads split the output
// rows that feed the input row into 256/R interleaved parts, reduced through LDS, so
// the 32-wide head (x8: ~15x15 contributing pixels per input pixel) runs on B*R
// blocks rather than B*R*R/256 (64 blocks at bs16: 70 us -> a few us).
// All heads in one launch (blocks [0, B*R0) for head 0, then B*R1 for head 1, ...): one
// launch instead of one per head (each a few us of latency-bound work); per block the same
// arithmetic, so dh is unchanged.
struct SplitSet {
    float* dh[4];
    int res[4];
    int n;
};
__device__ __forceinline__ void head_split_bwd_block(const float* dl, int H, int W, int nc,
                                                     float* dh, int R, int blk) {
    __shared__ float red[256];
    const int b = blk / R, iy = blk % R, tid = threadIdx.x;
    const int parts = R < 256 ? 256 / R : 1;
    const int part = R < 256 ? tid / R : 0, lane = R < 256 ? tid % R : tid;
    int ylo, yhi;
    ac_range_tight(iy, R, H, ylo, yhi);
    for (int k = 0; k < nc; ++k) {
        const float* src = dl + ((size_t)b * nc + k) * H * W;
        for (int ix0 = 0; ix0 < R; ix0 += 256) {
            const int ix = ix0 + lane;
            float s = 0.f;
            if (part < parts && ix < R) {
                if (R == H) {
                    if (part == 0) s = src[(size_t)iy * W + ix];
                } else {
                    int xlo, xhi;
                    ac_range_tight(ix, R, W, xlo, xhi);
                    for (int oy = ylo + part; oy <= yhi; oy += parts) {
                        const float wy = ac_weight(oy, iy, R, H);
                        if (wy == 0.f) continue;
                        const float* row = src + (size_t)oy * W;
                        float r = 0.f;
                        for (int ox = xlo; ox <= xhi; ++ox) {
                            const float wx = ac_weight(ox, ix, R, W);
                            if (wx != 0.f) r = fmaf(wx, row[ox], r);
                        }
                        s = fmaf(wy, r, s);
                    }
                }
            }
            if (parts > 1) {
                __syncthreads();  // previous channel's reads of red are done
                red[tid] = s;
                __syncthreads();
                if (part == 0)
                    for (int q = 1; q < parts; ++q) s += red[q * R + lane];
            }
            if (part == 0 && ix < R) dh[(((size_t)b * R + iy) * R + ix) * nc + k] = s;
        }
    }
}
__global__ void __launch_bounds__(256) head_split_bwd_kernel(const float* dl, int B, int H,
                                                             int W, int nc, SplitSet hs) {
    int blk = blockIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j >= hs.n) break;
        const int nb = B * hs.res[j];
        if (blk < nb) {
            head_split_bwd_block(dl, H, W, nc, hs.dh[j], hs.res[j], blk);
            return;
        }
        blk -= nb;
    }
}

// da (+)= dh @ w ; per-block partials of dW = dh^T act and db = sum dh.  Compile-time
// class count NC and 64-channel slices CJ keep the accumulators in registers (runtime
// bounds put them in scratch); two pixels per iteration keep 2x the loads in flight.
// BNB: also the BatchNorm-backward partials of da (x is that BatchNorm's input y and
// (sc, sh) its affine, already loaded here: the fusion costs no memory traffic); same
// block plan, so nslots = the block count (ugpg_head_bwd_bnb_slots).
template <int NC, int CJ, bool BNB>
__global__ void __launch_bounds__(256) head_bwd_kernel(YRef x, const float* sc,
                                                       const float* sh, int64_t npix, int C,
                                                       const float* w, int nc, const float* dh,
                                                       float* da, int acc_da, int64_t ppb,
                                                       float* part, int nblk, BnbArgs bnb) {
    const int tid = threadIdx.x, l16 = tid & 15, slot = tid >> 4;
    BnbAcc bacc[BNB ? CJ : 1];
    if constexpr (BNB)
#pragma unroll
        for (int j = 0; j < CJ; ++j) bacc[j].init(bnb, l16 * 4 + 64 * j);
    f32x4 gw[NC][CJ];
    float gb[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        gb[k] = 0.f;
#pragma unroll
        for (int j = 0; j < CJ; ++j) gw[k][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 wk[NC][CJ];
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
        for (int j = 0; j < CJ; ++j)
            wk[k][j] = *reinterpret_cast<const f32x4*>(w + (size_t)k * C + l16 * 4 + 64 * j);
    const int64_t p0 = blockIdx.x * ppb, p1 = min(npix, p0 + ppb);
    auto pixel = [&](int64_t p, const float (&d)[NC], const f32x4 (&xv)[CJ]) {
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            const int c = l16 * 4 + 64 * j;
            const f32x4 v = act_apply4(xv[j], sc, sh, c);
            f32x4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                g += d[k] * wk[k][j];
                gw[k][j] += d[k] * v;
            }
            f32x4* dst = reinterpret_cast<f32x4*>(da + p * C + c);
            if (acc_da & 1) g += *dst;
            if (!(acc_da & UGPG_HEAD_DA_DEFERRED)) *dst = g;  // (deferred: the apply recomputes it)
            if constexpr (BNB) bacc[j].add(g, xv[j]);
        }
        if (l16 == 0)
#pragma unroll
            for (int k = 0; k < NC; ++k) gb[k] += d[k];
    };
    int64_t p = p0 + slot;
    for (; p + 16 < p1; p += 32) {
        float d0[NC], d1[NC];
        f32x4 x0[CJ], x1[CJ];
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            d0[k] = dh[p * NC + k];
            d1[k] = dh[(p + 16) * NC + k];
        }
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            x0[j] = x.ld4(p * C + l16 * 4 + 64 * j);
            x1[j] = x.ld4((p + 16) * C + l16 * 4 + 64 * j);
        }
        pixel(p, d0, x0);
        pixel(p + 16, d1, x1);
    }
    for (; p < p1; p += 16) {
        float d0[NC];
        f32x4 x0[CJ];
#pragma unroll
        for (int k = 0; k < NC; ++k) d0[k] = dh[p * NC + k];
#pragma unroll
        for (int j = 0; j < CJ; ++j)
            x0[j] = x.ld4(p * C + l16 * 4 + 64 * j);
        pixel(p, d0, x0);
    }
    __shared__ f32x4 red[256];
    __shared__ float redb[16];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            red[tid] = gw[k][j];
            if (l16 == 0) redb[slot] = gb[k];
            __syncthreads();
            if (slot == 0) {
                f32x4 s = red[l16];
                for (int q = 1; q < 16; ++q) s += red[q * 16 + l16];
                float* dst = part + ((size_t)blockIdx.x * NC + k) * (C + 1) + l16 * 4 + 64 * j;
                dst[0] = s.x;
                dst[1] = s.y;
                dst[2] = s.z;
                dst[3] = s.w;
                if (l16 == 0 && j == 0) {
                    float sb = 0.f;
                    for (int q = 0; q < 16; ++q) sb += redb[q];
                    part[((size_t)blockIdx.x * NC + k) * (C + 1) + C] = sb;
                }
            }
            __syncthreads();
        }
    }
    if constexpr (BNB) {
        // BatchNorm-backward partials: per 64-channel slice, the 16 pixel slots in order
        __shared__ f32x4 rb[3][256];
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
            rb[0][tid] = bacc[j].sg;
            rb[1][tid] = bacc[j].sgx;
            rb[2][tid] = bacc[j].sx;
            __syncthreads();
            if (slot == 0) {
                f32x4 a0 = rb[0][l16], a1 = rb[1][l16], a2 = rb[2][l16];
                for (int q = 1; q < 16; ++q) {
                    a0 += rb[0][q * 16 + l16];
                    a1 += rb[1][q * 16 + l16];
                    a2 += rb[2][q * 16 + l16];
                }
                const int c = l16 * 4 + 64 * j;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    bnb.part[(size_t)(c + k) * nblk + blockIdx.x] = a0[k];
                    bnb.part[((size_t)C + c + k) * nblk + blockIdx.x] = a1[k];
                    bnb.part[((size_t)2 * C + c + k) * nblk + blockIdx.x] = a2[k];
                }
            }
            __syncthreads();
        }
    }
}

// fixed-order block tree: thread i sums i, i+256, ... then an LDS tree
__device__ __forceinline__ double block_tree_sum(double v) {
    __shared__ double t[256];
    t[threadIdx.x] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) t[threadIdx.x] += t[threadIdx.x + s];
        __syncthreads();
    }
    const double r = t[0];
    __syncthreads();
    return r;
}

// Block = 16 consecutive outputs x 64 partial-groups: thread (g, l) sums partial blocks
// g, g+64, ... (up to 16 for the 1,024-block head backward of a 256^2 head; 16 groups of 64
// serial loads each held it at 7 us) then a fixed 64-way combine in order.
__global__ void __launch_bounds__(1024) head_bwd_finalize_kernel(const float* part, int nblk, int nc,
                                                                 int C, float* dw, float* db) {
    __shared__ double red[64][16];
    const int total = nc * (C + 1);
    const int l = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int e = blockIdx.x * 16 + l;
    double s = 0;
    if (e < total) {
        int i = g;
        for (; i + 192 < nblk; i += 256) {
            const float a0 = part[(size_t)i * total + e], a1 = part[(size_t)(i + 64) * total + e];
            const float a2 = part[(size_t)(i + 128) * total + e];
            const float a3 = part[(size_t)(i + 192) * total + e];
            s += a0;
            s += a1;
            s += a2;
            s += a3;
        }
        for (; i < nblk; i += 64) s += part[(size_t)i * total + e];
    }
    red[g][l] = s;
    __syncthreads();
    if (g == 0 && e < total) {
        for (int q = 1; q < 64; ++q) s += red[q][l];
        const int k = e / (C + 1), c = e % (C + 1);
        if (c < C) dw[(size_t)k * C + c] = (float)s;
        else if (db) db[k] = (float)s;
    }
}

// ------------------------------------------------------------- UG loss
__device__ __forceinline__ void block_sum2(double& a, double& b) {
    __shared__ double sa[4], sb[4];
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        sa[wave] = a;
        sb[wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = sa[0] + sa[1] + sa[2] + sa[3];
        b = sb[0] + sb[1] + sb[2] + sb[3];
    }
}

__device__ __forceinline__ float bce_pixel(float x, float t, float pw) {
    const float lw = 1.0f + (pw - 1.0f) * t;
    const float sp = log1pf(expf(-fabsf(x))) - fminf(x, 0.0f);  // softplus(-x) = -log_sigmoid(x)
    return (1.0f - t) * x + lw * sp;
}

__device__ __forceinline__ float umap_at(const float* u, int64_t i, int C, int HW, int Cu) {
    if (!u) return 0.f;
    if (Cu == C) return u[i];
    const int64_t p = i % HW, b = i / ((int64_t)C * HW);
    return u[b * HW + p];
}

__global__ void __launch_bounds__(256) ug_loss_fwd_kernel(const float* x, const float* t,
                                                          const float* u, int64_t n, int C, int HW,
                                                          int Cu, const float* pwp, float alpha,
                                                          const float* pixel_loss,
                                                          double* part) {
    const float pw = pwp ? pwp[0] : 1.0f;
    double sp = 0, sw = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float pl = pixel_loss ? pixel_loss[i] : bce_pixel(x[i], t[i], pw);
        sp += pl;
        sw += pl * (1.0f + alpha * umap_at(u, i, C, HW, Cu));
    }
    block_sum2(sp, sw);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sp;
        part[2 * blockIdx.x + 1] = sw;
    }
}

__global__ void __launch_bounds__(256) ug_loss_finalize_kernel(const double* part, int nblk,
                                                               int64_t n, int has_u, float* out) {
    double sp = 0, sw = 0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        sp += part[2 * i];
        sw += part[2 * i + 1];
    }
    sp = block_tree_sum(sp);
    sw = block_tree_sum(sw);
    if (threadIdx.x == 0) {
        out[0] = (float)((has_u ? sw : sp) / (double)n);
        out[1] = (float)(sp / (double)n);
    }
}

__global__ void ug_loss_bwd_kernel(const float* x, const float* t, const float* u, int64_t n,
                                   int C, int HW, int Cu, const float* pwp, float alpha,
                                   const float* gout, float* dx, int generic) {
    const float pw = pwp ? pwp[0] : 1.0f;
    const float g = gout[0] / (float)n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float w = 1.0f + alpha * umap_at(u, i, C, HW, Cu);
        if (generic) {
            dx[i] = g * w;
        } else {
            const float tt = t[i], xx = x[i];
            const float lw = 1.0f + (pw - 1.0f) * tt;
            const float sneg = 1.0f / (1.0f + expf(xx));  // sigmoid(-x)
            dx[i] = g * w * ((1.0f - tt) - lw * sneg);
        }
    }
}

// ------------------------------------------------------------- metrics
__global__ void __launch_bounds__(256) seg_metrics_kernel(const float* x, const float* t, int HW,
                                                          int nbps, float* part) {
    const int b = blockIdx.y;
    float si = 0, sp = 0, st = 0, sw = 0;
    const int per = (HW + nbps - 1) / nbps;
    const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
    for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const size_t i = (size_t)b * HW + p;
        const float pr = sigmoidf_(x[i]) > 0.5f ? 1.0f : 0.0f;
        const float tv = t[i];
        si += pr * tv;
        sp += pr;
        st += tv;
        sw += (pr != truncf(tv)) ? 1.0f : 0.0f;
    }
    si = wave_sum(si);
    sp = wave_sum(sp);
    st = wave_sum(st);
    sw = wave_sum(sw);
    __shared__ float red[4][4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        red[wave][0] = si;
        red[wave][1] = sp;
        red[wave][2] = st;
        red[wave][3] = sw;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        part[((size_t)b * nbps + blockIdx.x) * 4 + threadIdx.x] = s;
    }
}

__global__ void __launch_bounds__(256) seg_metrics_finalize_kernel(const float* part, int B,
                                                                   int nbps, int64_t npix,
                                                                   float* out) {
    // per-sample counts (exact in fp32), one thread per (sample, quantity)
    __shared__ float cnt[1024];
    for (int e = threadIdx.x; e < B * 4; e += 256) {
        const int b = e >> 2, q = e & 3;
        // eight independent chains (integer-valued partials below 2^24: exact in any order)
        float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < nbps; k0 += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (k0 + j < nbps) s8[j] += part[((size_t)b * nbps + k0 + j) * 4 + q];
        cnt[e] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float dsum = 0.f;
        double wrong = 0;
        for (int b = 0; b < B; ++b) {
            dsum += (2.0f * cnt[4 * b] + 1.0f) / (cnt[4 * b + 1] + cnt[4 * b + 2] + 1.0f);
            wrong += cnt[4 * b + 3];
        }
        out[0] = dsum / (float)B;
        out[1] = (float)(1.0 - wrong / (double)npix);
        out[2] = (float)wrong;
    }
}

// ------------------------------------------------------------- inference / evaluation
// MoNuSegTester.calculate_metrics / predict_image (MoNuSegImprove/test_monuseg.py:164-297):
// per-sample counts of pred = sigmoid(x) > 0.5 against a ground-truth mask, then the six
// metrics in float32 exactly as numpy evaluates them on float32 arrays (eps 1e-8).
__global__ void __launch_bounds__(256) seg_eval_part_kernel(const float* x, const float* t, int HW,
                                                            int nbps, double* part) {
    const int b = blockIdx.y;
    double stp = 0, sp = 0, st = 0, ss = 0;
    const int per = (HW + nbps - 1) / nbps;
    const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
    for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const size_t i = (size_t)b * HW + p;
        const float pr = sigmoidf_(x[i]);
        const float pm = pr > 0.5f ? 1.0f : 0.0f;
        const float tv = t[i];
        stp += (double)(pm * tv);
        sp += pm;
        st += tv;
        ss += pr;
    }
    stp = wave_sum_d(stp);
    sp = wave_sum_d(sp);
    st = wave_sum_d(st);
    ss = wave_sum_d(ss);
    __shared__ double red[4][4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        red[wave][0] = stp;
        red[wave][1] = sp;
        red[wave][2] = st;
        red[wave][3] = ss;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const double v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                         red[3][threadIdx.x];
        part[((size_t)b * nbps + blockIdx.x) * 4 + threadIdx.x] = v;
    }
}

__global__ void seg_eval_finalize_kernel(const double* part, int B, int nbps, int HW, float* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double c[4] = {0, 0, 0, 0};
    for (int k = 0; k < nbps; ++k)
        for (int q = 0; q < 4; ++q) c[q] += part[((size_t)b * nbps + k) * 4 + q];
    // float32 arithmetic in the reference's order (numpy on float32 arrays; python
    // scalars are weak under NEP 50, so eps and len() enter as float32)
    const float eps = 1e-8f;
    const float tp = (float)c[0], sp = (float)c[1], st = (float)c[2];
    const float fp = sp - tp, fn = st - tp;
    const float tn = (((float)HW - tp) - fp) - fn;
    float* o = out + (size_t)b * 8;
    o[0] = (tp + eps) / (((tp + fp) + fn) + eps);
    o[1] = (2.0f * tp + eps) / (((2.0f * tp + fp) + fn) + eps);
    o[2] = ((tp + tn) + eps) / ((((tp + tn) + fp) + fn) + eps);
    o[3] = (tp + eps) / ((tp + fp) + eps);
    o[4] = (tp + eps) / ((tp + fn) + eps);
    o[5] = (tn + eps) / ((tn + fp) + eps);
    o[6] = (float)(c[3] / (double)HW);  // confidence = mean probability
    o[7] = tp;
}

// mask = nearest-resize(sigmoid(x) > 0.5) to (Ho, Wo)  (test_monuseg.py:188-195)
__global__ void predict_mask_kernel(const float* x, int B, int H, int W, float* mask, int Ho,
                                    int Wo) {
    const int64_t total = (int64_t)B * Ho * Wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int ox = (int)(i % Wo);
        const int64_t r = i / Wo;
        const int oy = (int)(r % Ho);
        const int64_t b = r / Ho;
        const float v = x[((size_t)b * H + nearest_src(oy, H, Ho)) * W + nearest_src(ox, W, Wo)];
        mask[i] = sigmoidf_(v) > 0.5f ? 1.0f : 0.0f;
    }
}

// ---- data-parallel metrics (SURVEY §5 "metrics all-reduced under DP")
// A rank's metrics buffer m[0..n) holds per-rank means (bit i of avg_mask), counts
// (summed as is) and one (mean, unbiased std) pair at [ip, ip+1) over n_stat values.
// pack -> double sums[n + 2] (the pair as n*mean and M2 + n*mean^2, then n_stat and a
// rank count of 1); after a SUM all-reduce, unpack writes the global metrics back.
__global__ void metrics_pack_kernel(const float* m, int n, int ip, double n_stat, double* sums) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        double v = m[i];
        if (ip >= 0 && i == ip) {
            v = n_stat * (double)m[ip];
        } else if (ip >= 0 && i == ip + 1) {
            const double mu = m[ip], sd = m[ip + 1];
            v = (n_stat > 1 ? sd * sd * (n_stat - 1) : 0.0) + n_stat * mu * mu;
        }
        sums[i] = v;
    }
    if (threadIdx.x == 0) {
        sums[n] = n_stat;
        sums[n + 1] = 1.0;
    }
}

__global__ void metrics_unpack_kernel(const double* sums, int n, int ip, unsigned avg_mask,
                                      float* m) {
    const double ranks = sums[n + 1], N = sums[n];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        double v = sums[i];
        if (ip >= 0 && i == ip) {
            v = N > 0 ? sums[ip] / N : 0.0;
        } else if (ip >= 0 && i == ip + 1) {
            const double mu = N > 0 ? sums[ip] / N : 0.0;
            const double M2 = sums[ip + 1] - N * mu * mu;
            v = N > 1 ? sqrt(fmax(M2, 0.0) / (N - 1)) : 0.0;
        } else if (i < 32 && ((avg_mask >> i) & 1u)) {
            v /= ranks;
        }
        m[i] = (float)v;
    }
}

__global__ void __launch_bounds__(256) mean_std_part_kernel(const float* x, int64_t n,
                                                            int64_t per, double* part) {
    const int64_t p0 = blockIdx.x * per, p1 = min(n, p0 + per);
    double s = 0;
    for (int64_t i = p0 + threadIdx.x; i < p1; i += blockDim.x) s += x[i];
    double dummy = 0;
    block_sum2(s, dummy);
    __shared__ double mu_s;
    if (threadIdx.x == 0) mu_s = s / (double)(p1 - p0);
    __syncthreads();
    const double mu = mu_s;
    double q = 0;
    for (int64_t i = p0 + threadIdx.x; i < p1; i += blockDim.x) {
        const double d = x[i] - mu;
        q += d * d;
    }
    dummy = 0;
    __syncthreads();
    block_sum2(q, dummy);
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = (double)(p1 - p0);
        part[3 * blockIdx.x + 1] = mu;
        part[3 * blockIdx.x + 2] = q;
    }
}

__global__ void __launch_bounds__(256) mean_std_finalize_kernel(const double* part, int nblk,
                                                                float* out) {
    // Chan merge: strided per thread, then a fixed LDS tree
    __shared__ double sn[256], sm[256], sq[256];
    double n = 0, mu = 0, M = 0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        const double nb = part[3 * i];
        if (nb <= 0) continue;
        const double nn = n + nb, d = part[3 * i + 1] - mu;
        mu += d * nb / nn;
        M += part[3 * i + 2] + d * d * n * nb / nn;
        n = nn;
    }
    sn[threadIdx.x] = n;
    sm[threadIdx.x] = mu;
    sq[threadIdx.x] = M;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const double na = sn[threadIdx.x], nb = sn[threadIdx.x + s];
            if (nb > 0) {
                const double nn = na + nb, d = sm[threadIdx.x + s] - sm[threadIdx.x];
                sm[threadIdx.x] += d * nb / nn;
                sq[threadIdx.x] += sq[threadIdx.x + s] + d * d * na * nb / nn;
                sn[threadIdx.x] = nn;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = (float)sm[0];
        out[1] = (float)(sn[0] > 1 ? sqrt(sq[0] / (sn[0] - 1)) : (double)NAN);
    }
}

// ------------------------------------------------------------- RMSprop
__global__ void rmsprop_kernel(float* p, const float* g, float* v, int64_t n, float lr, float alpha,
                               float eps, float wd, float gs) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float pv = p[i];
        float gv = g[i];
        if (gs != 1.0f) gv *= gs;
        if (wd != 0.0f) gv = gv + wd * pv;
        const float sa = v[i] * alpha + (1.0f - alpha) * (gv * gv);
        v[i] = sa;
        p[i] = pv + (-lr) * (gv / (sqrtf(sa) + eps));
    }
}

__global__ void rmsprop4_kernel(f32x4* p, const f32x4* g, f32x4* v, int64_t n4, float lr,
                                float alpha, float eps, float wd, float gs) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const f32x4 pv = p[i];
        f32x4 gv = g[i], sv = v[i], out;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float gg = gv[k];
            if (gs != 1.0f) gg *= gs;
            if (wd != 0.0f) gg = gg + wd * pv[k];
            const float sa = sv[k] * alpha + (1.0f - alpha) * (gg * gg);
            sv[k] = sa;
            out[k] = pv[k] + (-lr) * (gg / (sqrtf(sa) + eps));
        }
        v[i] = sv;
        p[i] = out;
    }
}

// ------------------------------------------------------------- Herlev head
__global__ void avgpool_fwd_kernel(YRef x, const float* sc, const float* sh, int B, int HW,
                                   int C, float* out) {
    const int64_t total = (int64_t)B * C / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % (C / 4)) * 4, b = (int)(i / (C / 4));
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        for (int p = 0; p < HW; ++p)
            s += act_apply4(x.ld4(((size_t)b * HW + p) * C + c), sc, sh, c);
        *reinterpret_cast<f32x4*>(out + (size_t)b * C + c) = s / (float)HW;
    }
}

__global__ void avgpool_bwd_kernel(const float* dout, int B, int HW, int C, float* da, int acc) {
    const int64_t total = (int64_t)B * HW * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int b = (int)(i / ((int64_t)HW * C));
        const float v = dout[(size_t)b * C + c] / (float)HW;
        da[i] = acc ? da[i] + v : v;
    }
}

__global__ void linear_fwd_kernel(const float* x, const float* w, const float* b, int M, int N,
                                  int K, int relu, float* y) {
    // one wave per output element, lanes split K
    const int lane = threadIdx.x & 63;
    const int64_t total = (int64_t)M * N;
    for (int64_t o = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; o < total;
         o += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int m = (int)(o / N), n = (int)(o % N);
        float s = 0.f;
        for (int k = lane; k < K; k += 64) s += x[(size_t)m * K + k] * w[(size_t)n * K + k];
        s = wave_sum(s);
        if (lane == 0) {
            s += b ? b[n] : 0.f;
            y[o] = relu ? fmaxf(s, 0.f) : s;
        }
    }
}

__global__ void linear_bwd_dx_kernel(const float* w, const float* dy, int M, int N, int K,
                                     float* dx) {
    const int64_t total = (int64_t)M * K;
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(o / K), k = (int)(o % K);
        float s = 0.f;
        for (int n = 0; n < N; ++n) s += dy[(size_t)m * N + n] * w[(size_t)n * K + k];
        dx[o] = s;
    }
}

__global__ void linear_bwd_dw_kernel(const float* x, const float* dy, int M, int N, int K,
                                     float* dw, float* db) {
    const int64_t total = (int64_t)N * K;
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(o / K), k = (int)(o % K);
        float s = 0.f;
        for (int m = 0; m < M; ++m) s += dy[(size_t)m * N + n] * x[(size_t)m * K + k];
        dw[o] = s;
        if (db && k == 0) {
            float t = 0.f;
            for (int m = 0; m < M; ++m) t += dy[(size_t)m * N + n];
            db[n] = t;
        }
    }
}

__global__ void relu_bwd_kernel(const float* y, const float* dy, float* dx, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

__global__ void mul_kernel(const float* x, const float* m, float* y, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = x[i] * m[i];
}

namespace {
// (the reductions below: 4 elements per thread, up to 1,024 blocks -- at 16 per thread the
// bs16 x 256^2 loss, metrics and U statistics ran on 256 blocks, latency-bound: 11-21 us)
int loss_nblk(int64_t n) {
    int64_t b = cdiv(n, 256 * 4);
    if (b > 1024) b = 1024;
    return (int)(b < 1 ? 1 : b);
}
#ifndef HEAD_BWD_PPB_MIN
#define HEAD_BWD_PPB_MIN 64
#endif
// blocks of the head backward: at least 64 pixels each (4 per slot) up to 1,024 blocks -- the
// 32^2 and 64^2 heads of a bs16 step (16k / 65k pixels) then fill the chip (with 256 pixels
// per block the 32^2 head ran on 64 blocks: 50 us for 12 MB)
int head_nblk(int64_t npix, int64_t& ppb) {
    int64_t b = cdiv(npix, HEAD_BWD_PPB_MIN);
    if (b > 1024) b = 1024;
    if (b < 1) b = 1;
    ppb = cdiv(npix, b);
    return (int)cdiv(npix, ppb);
}
int metrics_nbps(int HW) {
    int n = (int)cdiv(HW, 1024);
    return n < 1 ? 1 : (n > 64 ? 64 : n);
}
int ms_nblk(int64_t n, int64_t& per) {
    int64_t b = cdiv(n, 1024);
    if (b > 1024) b = 1024;
    if (b < 1) b = 1;
    per = cdiv(n, b);
    return (int)cdiv(n, per);
}
}  // namespace
}  // namespace ugpg

using namespace ugpg;

#define UGPG_REQUIRE(cond, name)                         \
    do {                                                 \
        if (!(cond)) {                                   \
            set_error("%s: invalid argument (%s)", name, #cond); \
            return UGPG_ERR_INVALID;                     \
        }                                                \
    } while (0)

extern "C" int ugpg_maxpool2_fwd(ugpg_src_t s, int B, int H, int W, float* out, void* out_bf16,
                                 uint8_t* am, void* stream) {
    UGPG_REQUIRE((s.data || s.data_bf16) && (out || out_bf16) && am && s.C % 4 == 0 && H >= 2 &&
                     W >= 2,
                 "maxpool2_fwd");
    const int64_t total8 = (int64_t)B * (H / 2) * (W / 2) * (s.C / 8);
    if (!s.data && !out && s.C % 8 == 0 && 256 % (s.C / 8) == 0 &&
        total8 + 4 * (int64_t)stream_grid(cdiv(total8, (int64_t)4)) * 256 < (int64_t(1) << 32)) {
        // bf16 in and out: 16-byte accesses (32-bit unit indices)
        hipLaunchKernelGGL(maxpool2_fwd16_kernel, dim3(stream_grid(cdiv(total8, (int64_t)4))), dim3(256), 0,
                           as_stream(stream), static_cast<const __bf16*>(s.data_bf16), s.scale,
                           s.shift, B, H, W, s.C, static_cast<__bf16*>(out_bf16), am);
        return check_launch("maxpool2_fwd");
    }
    const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (s.C / 4);
    hipLaunchKernelGGL(maxpool2_fwd_kernel<false>, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), yref(s), s.scale, s.shift, B, H, W, s.C, out,
                       static_cast<__bf16*>(out_bf16), am);
    return check_launch("maxpool2_fwd");
}

extern "C" int ugpg_maxpool2_bwd(const float* dout, const uint8_t* am, int B, int H, int W, int C,
                                 float* din, int acc, void* stream) {
    UGPG_REQUIRE(dout && am && din && C % 4 == 0, "maxpool2_bwd");
    const int64_t total = (int64_t)B * H * W * (C / 4);
    hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), dout, am, B, H, W, C, din, acc);
    return check_launch("maxpool2_bwd");
}

static bool bnb_args(const ugpg_bnb_t* d, int64_t npix, int C, BnbArgs& b) {
    if (!d || (!d->y && !d->y_bf16) || !d->mean || !d->invstd || !d->scale || !d->shift || !d->part ||
        d->nslots != ugpg_bnb_slots(npix, C) || C % 4 || C > 1024)
        return false;
    b.y = yref(d->y, d->y_bf16);
    b.mean = d->mean;
    b.invstd = d->invstd;
    b.scale = d->scale;
    b.shift = d->shift;
    b.part = d->part;
    b.nblk = d->nslots;
    b.ppb = cdiv(npix, (int64_t)d->nslots);
    return true;
}

extern "C" int ugpg_maxpool2_bwd_bnb(const float* dout, const uint8_t* am, int B, int H, int W,
                                     int C, float* din, int acc, const ugpg_bnb_t* bnb,
                                     void* stream) {
    BnbArgs b;
    UGPG_REQUIRE(dout && am && din && B > 0 && H > 0 && W > 0 &&
                     (int64_t)B * H * W < (int64_t(1) << 31) && bnb_args(bnb, (int64_t)B * H * W, C, b),
                 "maxpool2_bwd_bnb");
    hipLaunchKernelGGL(maxpool2_bwd_bnb_kernel<true>, dim3(b.nblk), dim3(256), 0,
                       as_stream(stream), dout, am, B, H, W, C, din, acc, b);
    return check_launch("maxpool2_bwd_bnb");
}

extern "C" int ugpg_maxpool2_bwd_partials(const float* dout, const uint8_t* am, int B, int H,
                                          int W, int C, const float* din_base,
                                          const ugpg_bnb_t* bnb, void* stream) {
    BnbArgs b;
    UGPG_REQUIRE(dout && am && B > 0 && H > 0 && W > 0 &&
                     (int64_t)B * H * W < (int64_t(1) << 31) && bnb_args(bnb, (int64_t)B * H * W, C, b),
                 "maxpool2_bwd_partials");
    hipLaunchKernelGGL(maxpool2_bwd_bnb_kernel<false>, dim3(b.nblk), dim3(256), 0,
                       as_stream(stream), dout, am, B, H, W, C, const_cast<float*>(din_base),
                       din_base ? 1 : 0, b);
    return check_launch("maxpool2_bwd_partials");
}

extern "C" int ugpg_bilinear_nhwc_fwd(ugpg_src_t s, int B, int Hi, int Wi, float* out, int Ho,
                                      int Wo, void* out_bf16, void* stream) {
    UGPG_REQUIRE((s.data || s.data_bf16) && (out || out_bf16) && s.C % 4 == 0 && Ho > 0 && Wo > 0,
                 "bilinear_nhwc_fwd");
    UGPG_REQUIRE((int64_t)B * Ho < 65536, "bilinear_nhwc_fwd: shape");
    // a quarter of the row's quads in threads when that divides evenly (the kernel's
    // 4-quads-per-thread form), else one quad per thread
    if (!s.data && !out && s.C % 8 == 0 && 256 % (s.C / 8) == 0) {  // bf16 in and out: 16-byte accesses
        // one block per output row (its 2048-unit rows: 8 units per thread), more for wider rows
        const unsigned g8 = (unsigned)std::min<int64_t>(cdiv((int64_t)Wo * (s.C / 8), 2048), 64);
        hipLaunchKernelGGL(bilinear_nhwc_fwd16_kernel, dim3(g8, (unsigned)(B * Ho)), dim3(256), 0,
                           as_stream(stream), static_cast<const __bf16*>(s.data_bf16), s.scale,
                           s.shift, B, Hi, Wi, s.C, static_cast<__bf16*>(out_bf16), Ho, Wo);
        return check_launch("bilinear_nhwc_fwd");
    }
    const int64_t nq = (int64_t)Wo * (s.C / 4);
    const unsigned gx = nq % 1024 == 0 ? (unsigned)std::min<int64_t>(nq / 1024, 64)
                                       : (unsigned)std::min<int64_t>(cdiv(nq, 256), 64);
    hipLaunchKernelGGL(bilinear_nhwc_fwd_kernel, dim3(gx, (unsigned)(B * Ho)), dim3(256), 0,
                       as_stream(stream), yref(s), s.scale, s.shift, B, Hi, Wi, s.C, out,
                       out ? nullptr : static_cast<__bf16*>(out_bf16), Ho, Wo);
    return check_launch("bilinear_nhwc_fwd");
}

extern "C" int ugpg_bilinear_nhwc_bwd(const float* dout, int B, int Ho, int Wo, int C, float* din,
                                      int Hi, int Wi, int acc, void* stream) {
    UGPG_REQUIRE(dout && din && C % 4 == 0, "bilinear_nhwc_bwd");
    UGPG_REQUIRE((int64_t)B * Hi < 65536, "bilinear_nhwc_bwd: shape");
    const unsigned gx = (unsigned)std::min<int64_t>(cdiv((int64_t)Wi * (C / 4), 256), 64);
    hipLaunchKernelGGL(bilinear_nhwc_bwd_kernel, dim3(gx, (unsigned)(B * Hi)), dim3(256), 0,
                       as_stream(stream), dout, B, Ho, Wo, C, din, Hi, Wi, acc);
    return check_launch("bilinear_nhwc_bwd");
}

extern "C" int ugpg_bilinear_nhwc_bwd_bnb(const float* dout, int B, int Ho, int Wo, int C,
                                          float* din, int Hi, int Wi, int acc,
                                          const ugpg_bnb_t* bnb, void* stream) {
    BnbArgs b;
    // one workgroup (= partial slot) per input row; its threads keep their channels
    UGPG_REQUIRE(dout && din && B > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && C % 4 == 0 &&
                     C <= 1024 && 256 % (C / 4) == 0 && bnb && bnb->nslots == B * Hi &&
                     (bnb->y || bnb->y_bf16) && bnb->mean && bnb->invstd && bnb->scale && bnb->shift && bnb->part,
                 "bilinear_nhwc_bwd_bnb");
    b.y = yref(bnb->y, bnb->y_bf16);
    b.mean = bnb->mean;
    b.invstd = bnb->invstd;
    b.scale = bnb->scale;
    b.shift = bnb->shift;
    b.part = bnb->part;
    b.nblk = bnb->nslots;
    b.ppb = Wi;
    hipLaunchKernelGGL(bilinear_nhwc_bwd_bnb_kernel, dim3(b.nblk), dim3(256), 0,
                       as_stream(stream), dout, B, Ho, Wo, C, din, Hi, Wi, acc, b);
    return check_launch("bilinear_nhwc_bwd_bnb");
}

extern "C" int ugpg_cast_f32_bf16(const float* in, uint16_t* out, int64_t n, void* stream) {
    UGPG_REQUIRE(in && out && n >= 0, "cast_f32_bf16");
    if (n == 0) return UGPG_OK;
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream),
                       in, out, n);
    return check_launch("cast_f32_bf16");
}

extern "C" int ugpg_cast_bf16_f32(const uint16_t* in, float* out, int64_t n, void* stream) {
    UGPG_REQUIRE(in && out && n >= 0, "cast_bf16_f32");
    if (n == 0) return UGPG_OK;
    hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream),
                       in, out, n);
    return check_launch("cast_bf16_f32");
}

extern "C" int ugpg_resize_nchw(const float* in, int B, int C, int Hi, int Wi, float* out, int Ho,
                                int Wo, int mode, void* stream) {
    UGPG_REQUIRE(in && out && mode >= 0 && mode <= 2 && Ho > 0 && Wo > 0, "resize_nchw");
    const int64_t total = (int64_t)B * C * Ho * Wo;
    hipLaunchKernelGGL(resize_nchw_kernel, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), in, B * C, Hi, Wi, out, Ho, Wo, mode);
    return check_launch("resize_nchw");
}

extern "C" int ugpg_resize_nchw_bwd(const float* dout, int B, int C, int Ho, int Wo, float* din,
                                    int Hi, int Wi, void* stream) {
    UGPG_REQUIRE(dout && din && B > 0 && C > 0 && Ho > 0 && Wo > 0 && Hi > 0 && Wi > 0,
                 "resize_nchw_bwd");
    const int64_t total = (int64_t)B * C * Hi * Wi;
    hipLaunchKernelGGL(resize_nchw_bwd_kernel, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), dout, B * C, Ho, Wo, din, Hi, Wi);
    return check_launch("resize_nchw_bwd");
}

extern "C" int ugpg_nchw_to_nhwc(const float* in, int B, int C, int H, int W, float* out, int Cp,
                                 void* stream) {
    UGPG_REQUIRE(in && out && Cp >= C, "nchw_to_nhwc");
    const int64_t total = (int64_t)B * H * W;
    if (Cp % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0)
        hipLaunchKernelGGL(nchw_to_nhwc_kernel<true>, dim3(stream_grid(total)), dim3(256), 0,
                           as_stream(stream), in, B, C, H * W, out, Cp);
    else
        hipLaunchKernelGGL(nchw_to_nhwc_kernel<false>, dim3(stream_grid(total)), dim3(256), 0,
                           as_stream(stream), in, B, C, H * W, out, Cp);
    return check_launch("nchw_to_nhwc");
}

extern "C" int ugpg_nhwc_to_nchw(const float* in, int B, int C, int H, int W, int Cs, float* out,
                                 int acc, void* stream) {
    UGPG_REQUIRE(in && out && Cs >= C, "nhwc_to_nchw");
    const int64_t total = (int64_t)B * H * W * C;
    hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), in, B, C, H * W, Cs, out, acc);
    return check_launch("nhwc_to_nchw");
}

extern "C" int ugpg_head_fwd(ugpg_src_t s, int64_t npix, const float* w, const float* b, int nc,
                             float* h, void* stream) {
    UGPG_REQUIRE((s.data || s.data_bf16) && w && b && h && s.C % 64 == 0 && s.C <= 64 * HEAD_CJ_MAX && nc >= 1 &&
                     nc <= HEAD_NC_MAX,
                 "head_fwd");
    const dim3 grid(stream_grid(cdiv(npix, (int64_t)4) * 16));
    if (s.C == 64)
        hipLaunchKernelGGL(head_fwd8_kernel, dim3(stream_grid(cdiv(npix, (int64_t)4) * 8)), dim3(256), 0,
                           as_stream(stream), yref(s), s.scale, s.shift, npix, w, b, nc, h);
    else if (s.C == 128)
        hipLaunchKernelGGL(head_fwd_cj_kernel<2>, grid, dim3(256), 0, as_stream(stream), yref(s),
                           s.scale, s.shift, npix, w, b, nc, h);
    else if (s.C == 256)
        hipLaunchKernelGGL(head_fwd_cj_kernel<4>, grid, dim3(256), 0, as_stream(stream), yref(s),
                           s.scale, s.shift, npix, w, b, nc, h);
    else
        hipLaunchKernelGGL(head_fwd_kernel, dim3(stream_grid(npix * 16)), dim3(256), 0,
                           as_stream(stream), yref(s), s.scale, s.shift, npix, s.C, w, b, nc, h);
    return check_launch("head_fwd");
}

extern "C" int ugpg_heads_combine(const float* const* h, const int* hres, int n, int B, int H,
                                  int W, int nc, float* logits, void* stream) {
    UGPG_REQUIRE(h && hres && n >= 1 && n <= 4 && logits && H == W, "heads_combine");
    HeadSet hs;
    hs.n = n;
    for (int i = 0; i < 4; ++i) {
        hs.h[i] = i < n ? h[i] : nullptr;
        hs.res[i] = i < n ? hres[i] : 0;
    }
    const int64_t total = (int64_t)B * nc * H * W;
    if (W % 4 == 0)
        hipLaunchKernelGGL(heads_combine_kernel, dim3(stream_grid(total / 4)), dim3(256), 0,
                           as_stream(stream), hs, B, H, W, nc, logits);
    else
        hipLaunchKernelGGL(heads_combine1_kernel, dim3(stream_grid(total)), dim3(256), 0,
                           as_stream(stream), hs, B, H, W, nc, logits);
    return check_launch("heads_combine");
}

extern "C" int ugpg_heads_split_bwd(const float* dl, int B, int H, int W, int nc, float* const* dh,
                                    const int* hres, int n, void* stream) {
    UGPG_REQUIRE(dl && dh && hres && n >= 1 && H == W, "heads_split_bwd");
    UGPG_REQUIRE(n <= 4, "heads_split_bwd: at most 4 heads");
    SplitSet hs{};
    hs.n = n;
    int64_t blocks = 0;
    for (int i = 0; i < n; ++i) {
        UGPG_REQUIRE(hres[i] >= 1 && hres[i] <= H && dh[i], "heads_split_bwd: head resolution");
        hs.dh[i] = dh[i];
        hs.res[i] = hres[i];
        blocks += (int64_t)B * hres[i];
    }
    hipLaunchKernelGGL(head_split_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       as_stream(stream), dl, B, H, W, nc, hs);
    return check_launch("heads_split_bwd");
}

extern "C" size_t ugpg_head_bwd_workspace(int64_t npix, int C, int nc) {
    int64_t ppb;
    const int nblk = head_nblk(npix, ppb);
    return (size_t)nblk * nc * (C + 1) * sizeof(float);
}

extern "C" int ugpg_head_bwd_bnb_slots(int64_t npix) {
    int64_t ppb;
    return npix > 0 ? head_nblk(npix, ppb) : 0;
}

static int head_bwd_common(ugpg_src_t s, int64_t npix, const float* w, int nc, const float* dh,
                           float* dw, float* db, float* da, int acc_da, void* ws,
                           size_t ws_bytes, const ugpg_bnb_t* bnbd, void* stream);

extern "C" int ugpg_head_bwd(ugpg_src_t s, int64_t npix, const float* w, int nc, const float* dh,
                             float* dw, float* db, float* da, int acc_da, void* ws,
                             size_t ws_bytes, void* stream) {
    return head_bwd_common(s, npix, w, nc, dh, dw, db, da, acc_da, ws, ws_bytes, nullptr, stream);
}

extern "C" int ugpg_head_bwd_bnb(ugpg_src_t s, int64_t npix, const float* w, int nc,
                                 const float* dh, float* dw, float* db, float* da, int acc_da,
                                 void* ws, size_t ws_bytes, const ugpg_bnb_t* bnb, void* stream) {
    UGPG_REQUIRE(bnb && bnb->y == s.data && bnb->y_bf16 == (s.data ? bnb->y_bf16 : s.data_bf16) &&
                     s.scale && bnb->nslots == ugpg_head_bwd_bnb_slots(npix),
                 "head_bwd_bnb");
    return head_bwd_common(s, npix, w, nc, dh, dw, db, da, acc_da, ws, ws_bytes, bnb, stream);
}

static int head_bwd_common(ugpg_src_t s, int64_t npix, const float* w, int nc, const float* dh,
                           float* dw, float* db, float* da, int acc_da, void* ws,
                           size_t ws_bytes, const ugpg_bnb_t* bnbd, void* stream) {
    const bool deferred = acc_da & UGPG_HEAD_DA_DEFERRED;
    UGPG_REQUIRE((s.data || s.data_bf16) && w && dh && dw && (da || (deferred && !(acc_da & 1))) &&
                     (!deferred || bnbd) && (acc_da & ~3) == 0 && s.C % 64 == 0 &&
                     s.C <= 64 * HEAD_CJ_MAX && nc >= 1 && nc <= HEAD_NC_MAX,
                 "head_bwd");
    BnbArgs bnb{};
    if (bnbd) {
        UGPG_REQUIRE(bnbd->mean && bnbd->invstd && bnbd->scale && bnbd->shift && bnbd->part,
                     "head_bwd_bnb");
        bnb.y = yref(bnbd->y, bnbd->y_bf16);
        bnb.mean = bnbd->mean;
        bnb.invstd = bnbd->invstd;
        bnb.scale = bnbd->scale;
        bnb.shift = bnbd->shift;
        bnb.part = bnbd->part;
        bnb.nblk = bnbd->nslots;
    }
    const size_t need = ugpg_head_bwd_workspace(npix, s.C, nc);
    if (!ws || ws_bytes < need) {
        set_error("head_bwd: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    int64_t ppb;
    const int nblk = head_nblk(npix, ppb);
    hipStream_t st = as_stream(stream);
    using K = void (*)(YRef, const float*, const float*, int64_t, int, const float*, int,
                       const float*, float*, int, int64_t, float*, int, BnbArgs);
#define HB(B_)                                                                              \
    {{head_bwd_kernel<1, 1, B_>, head_bwd_kernel<1, 2, B_>, head_bwd_kernel<1, 3, B_>,     \
      head_bwd_kernel<1, 4, B_>},                                                          \
     {head_bwd_kernel<2, 1, B_>, head_bwd_kernel<2, 2, B_>, head_bwd_kernel<2, 3, B_>,     \
      head_bwd_kernel<2, 4, B_>},                                                          \
     {head_bwd_kernel<3, 1, B_>, head_bwd_kernel<3, 2, B_>, head_bwd_kernel<3, 3, B_>,     \
      head_bwd_kernel<3, 4, B_>},                                                          \
     {head_bwd_kernel<4, 1, B_>, head_bwd_kernel<4, 2, B_>, head_bwd_kernel<4, 3, B_>,     \
      head_bwd_kernel<4, 4, B_>}}
    static const K table[2][HEAD_NC_MAX][HEAD_CJ_MAX] = {HB(false), HB(true)};
#undef HB
    hipLaunchKernelGGL(table[bnbd ? 1 : 0][nc - 1][s.C / 64 - 1], dim3(nblk), dim3(256), 0, st,
                       yref(s), s.scale, s.shift, npix, s.C, w, nc, dh, da, acc_da, ppb,
                       static_cast<float*>(ws), nblk, bnb);
    if (int e = check_launch("head_bwd")) return e;
    hipLaunchKernelGGL(head_bwd_finalize_kernel, dim3((unsigned)cdiv(nc * (s.C + 1), 16)), dim3(1024), 0,
                       st, static_cast<const float*>(ws), nblk, nc, s.C, dw, db);
    return check_launch("head_bwd_finalize");
}

extern "C" size_t ugpg_ug_loss_workspace(int64_t n) { return (size_t)loss_nblk(n) * 2 * sizeof(double); }

static int loss_fwd_common(const float* x, const float* t, const float* u, int B, int C, int HW,
                           int Cu, const float* pw, float alpha, const float* pl, float* out,
                           void* ws, size_t ws_bytes, void* stream, const char* name) {
    UGPG_REQUIRE(out && (pl || (x && t)) && (!u || Cu == 1 || Cu == C), name);
    const int64_t n = (int64_t)B * C * HW;
    const size_t need = ugpg_ug_loss_workspace(n);
    if (!ws || ws_bytes < need) {
        set_error("%s: workspace %zu < %zu", name, ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    const int nblk = loss_nblk(n);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(ug_loss_fwd_kernel, dim3(nblk), dim3(256), 0, st, x, t, u, n, C, HW, Cu, pw,
                       alpha, pl, static_cast<double*>(ws));
    if (int e = check_launch(name)) return e;
    hipLaunchKernelGGL(ug_loss_finalize_kernel, dim3(1), dim3(256), 0, st,
                       static_cast<const double*>(ws), nblk, n, u ? 1 : 0, out);
    return check_launch(name);
}

extern "C" int ugpg_ug_loss_fwd(const float* x, const float* t, const float* u, int B, int C,
                                int HW, int Cu, const float* pw, float alpha, float* out,
                                void* ws, size_t ws_bytes, void* stream) {
    return loss_fwd_common(x, t, u, B, C, HW, Cu, pw, alpha, nullptr, out, ws, ws_bytes, stream,
                           "ug_loss_fwd");
}

extern "C" int ugpg_ug_loss_bwd(const float* x, const float* t, const float* u, int B, int C,
                                int HW, int Cu, const float* pw, float alpha, const float* gout,
                                float* dx, void* stream) {
    UGPG_REQUIRE(x && t && gout && dx && (!u || Cu == 1 || Cu == C), "ug_loss_bwd");
    const int64_t n = (int64_t)B * C * HW;
    hipLaunchKernelGGL(ug_loss_bwd_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream),
                       x, t, u, n, C, HW, Cu, pw, alpha, gout, dx, 0);
    return check_launch("ug_loss_bwd");
}

extern "C" int ugpg_weighted_mean_fwd(const float* pl, const float* u, int B, int C, int HW,
                                      int Cu, float alpha, float* out, void* ws, size_t ws_bytes,
                                      void* stream) {
    UGPG_REQUIRE(pl, "weighted_mean_fwd");
    return loss_fwd_common(nullptr, nullptr, u, B, C, HW, Cu, nullptr, alpha, pl, out, ws,
                           ws_bytes, stream, "weighted_mean_fwd");
}

extern "C" int ugpg_weighted_mean_bwd(const float* u, int B, int C, int HW, int Cu, float alpha,
                                      const float* gout, float* dpl, void* stream) {
    UGPG_REQUIRE(gout && dpl && (!u || Cu == 1 || Cu == C), "weighted_mean_bwd");
    const int64_t n = (int64_t)B * C * HW;
    hipLaunchKernelGGL(ug_loss_bwd_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream),
                       nullptr, nullptr, u, n, C, HW, Cu, nullptr, alpha, gout, dpl, 1);
    return check_launch("weighted_mean_bwd");
}

extern "C" size_t ugpg_seg_metrics_workspace(int B) {
    return (size_t)B * 64 * 4 * sizeof(float);
}

extern "C" int ugpg_seg_metrics(const float* x, const float* t, int B, int HW, float* out, void* ws,
                                size_t ws_bytes, void* stream) {
    UGPG_REQUIRE(x && t && out && B > 0 && HW > 0, "seg_metrics");
    const int nbps = metrics_nbps(HW);
    const size_t need = (size_t)B * nbps * 4 * sizeof(float);
    if (!ws || ws_bytes < need) {
        set_error("seg_metrics: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(seg_metrics_kernel, dim3(nbps, B), dim3(256), 0, st, x, t, HW, nbps,
                       static_cast<float*>(ws));
    if (int e = check_launch("seg_metrics")) return e;
    hipLaunchKernelGGL(seg_metrics_finalize_kernel, dim3(1), dim3(256), 0, st,
                       static_cast<const float*>(ws), B, nbps, (int64_t)B * HW, out);
    return check_launch("seg_metrics_finalize");
}

extern "C" size_t ugpg_seg_eval_workspace(int B, int HW) {
    return (size_t)B * metrics_nbps(HW) * 4 * sizeof(double);
}

extern "C" int ugpg_seg_eval(const float* x, const float* t, int B, int HW, float* out, void* ws,
                             size_t ws_bytes, void* stream) {
    UGPG_REQUIRE(x && t && out && B > 0 && HW > 0, "seg_eval");
    const int nbps = metrics_nbps(HW);
    const size_t need = ugpg_seg_eval_workspace(B, HW);
    if (!ws || ws_bytes < need) {
        set_error("seg_eval: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(seg_eval_part_kernel, dim3(nbps, B), dim3(256), 0, st, x, t, HW, nbps,
                       static_cast<double*>(ws));
    if (int e = check_launch("seg_eval")) return e;
    hipLaunchKernelGGL(seg_eval_finalize_kernel, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, st,
                       static_cast<const double*>(ws), B, nbps, HW, out);
    return check_launch("seg_eval_finalize");
}

extern "C" int ugpg_predict_mask(const float* x, int B, int H, int W, float* mask, int Ho, int Wo,
                                 void* stream) {
    UGPG_REQUIRE(x && mask && B > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, "predict_mask");
    hipLaunchKernelGGL(predict_mask_kernel, dim3(stream_grid((int64_t)B * Ho * Wo)), dim3(256), 0,
                       as_stream(stream), x, B, H, W, mask, Ho, Wo);
    return check_launch("predict_mask");
}

extern "C" int ugpg_metrics_pack(const float* m, int n, int ip, double n_stat, double* sums,
                                 void* stream) {
    UGPG_REQUIRE(m && sums && n > 0 && n <= 32 && ip < n - 1 && n_stat >= 0, "metrics_pack");
    hipLaunchKernelGGL(metrics_pack_kernel, dim3(1), dim3(64), 0, as_stream(stream), m, n, ip,
                       n_stat, sums);
    return check_launch("metrics_pack");
}

extern "C" int ugpg_metrics_unpack(const double* sums, int n, int ip, unsigned avg_mask, float* m,
                                   void* stream) {
    UGPG_REQUIRE(m && sums && n > 0 && n <= 32 && ip < n - 1, "metrics_unpack");
    hipLaunchKernelGGL(metrics_unpack_kernel, dim3(1), dim3(64), 0, as_stream(stream), sums, n,
                       ip, avg_mask, m);
    return check_launch("metrics_unpack");
}

extern "C" size_t ugpg_mean_std_workspace(int64_t n) {
    int64_t per;
    return (size_t)ms_nblk(n, per) * 3 * sizeof(double);
}

extern "C" int ugpg_mean_std(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                             void* stream) {
    UGPG_REQUIRE(x && out && n > 0, "mean_std");
    int64_t per;
    const int nblk = ms_nblk(n, per);
    if (!ws || ws_bytes < (size_t)nblk * 3 * sizeof(double)) {
        set_error("mean_std: workspace too small");
        return UGPG_ERR_WORKSPACE;
    }
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(mean_std_part_kernel, dim3(nblk), dim3(256), 0, st, x, n, per,
                       static_cast<double*>(ws));
    if (int e = check_launch("mean_std")) return e;
    hipLaunchKernelGGL(mean_std_finalize_kernel, dim3(1), dim3(256), 0, st,
                       static_cast<const double*>(ws), nblk, out);
    return check_launch("mean_std_finalize");
}

extern "C" int ugpg_rmsprop_step(float* p, const float* g, float* v, int64_t n, float lr,
                                 float alpha, float eps, float wd, float gs, void* stream) {
    UGPG_REQUIRE(p && g && v && n >= 0, "rmsprop_step");
    if (n == 0) return UGPG_OK;
    hipStream_t st = as_stream(stream);
    const bool al = ((uintptr_t)p % 16 == 0) && ((uintptr_t)g % 16 == 0) && ((uintptr_t)v % 16 == 0);
    if (al && n % 4 == 0) {
        hipLaunchKernelGGL(rmsprop4_kernel, dim3(stream_grid(n / 4)), dim3(256), 0, st,
                           reinterpret_cast<f32x4*>(p), reinterpret_cast<const f32x4*>(g),
                           reinterpret_cast<f32x4*>(v), n / 4, lr, alpha, eps, wd, gs);
    } else {
        hipLaunchKernelGGL(rmsprop_kernel, dim3(stream_grid(n)), dim3(256), 0, st, p, g, v, n, lr,
                           alpha, eps, wd, gs);
    }
    return check_launch("rmsprop_step");
}

extern "C" int ugpg_avgpool_fwd(ugpg_src_t s, int B, int HW, float* out, void* stream) {
    UGPG_REQUIRE((s.data || s.data_bf16) && out && s.C % 4 == 0, "avgpool_fwd");
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(stream_grid((int64_t)B * s.C / 4)), dim3(256), 0,
                       as_stream(stream), yref(s), s.scale, s.shift, B, HW, s.C, out);
    return check_launch("avgpool_fwd");
}

extern "C" int ugpg_avgpool_bwd(const float* dout, int B, int HW, int C, float* da, int acc,
                                void* stream) {
    UGPG_REQUIRE(dout && da, "avgpool_bwd");
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(stream_grid((int64_t)B * HW * C)), dim3(256), 0,
                       as_stream(stream), dout, B, HW, C, da, acc);
    return check_launch("avgpool_bwd");
}

extern "C" int ugpg_linear_fwd(const float* x, const float* w, const float* b, int M, int N, int K,
                               int relu, float* y, void* stream) {
    UGPG_REQUIRE(x && w && y && M > 0 && N > 0 && K > 0, "linear_fwd");
    hipLaunchKernelGGL(linear_fwd_kernel, dim3(stream_grid((int64_t)M * N * 64)), dim3(256), 0,
                       as_stream(stream), x, w, b, M, N, K, relu, y);
    return check_launch("linear_fwd");
}

extern "C" int ugpg_linear_bwd(const float* x, const float* w, const float* dy, int M, int N,
                               int K, float* dx, float* dw, float* db, void* stream) {
    UGPG_REQUIRE(x && w && dy && dw, "linear_bwd");
    hipStream_t st = as_stream(stream);
    if (dx) {
        hipLaunchKernelGGL(linear_bwd_dx_kernel, dim3(stream_grid((int64_t)M * K)), dim3(256), 0,
                           st, w, dy, M, N, K, dx);
        if (int e = check_launch("linear_bwd_dx")) return e;
    }
    hipLaunchKernelGGL(linear_bwd_dw_kernel, dim3(stream_grid((int64_t)N * K)), dim3(256), 0, st,
                       x, dy, M, N, K, dw, db);
    return check_launch("linear_bwd_dw");
}

extern "C" int ugpg_relu_bwd(const float* y, const float* dy, float* dx, int64_t n,
                             void* stream) {
    UGPG_REQUIRE(y && dy && dx, "relu_bwd");
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream), y,
                       dy, dx, n);
    return check_launch("relu_bwd");
}

extern "C" int ugpg_mul(const float* x, const float* m, float* y, int64_t n, void* stream) {
    UGPG_REQUIRE(x && m && y, "mul");
    hipLaunchKernelGGL(mul_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream), x, m, y,
                       n);
    return check_launch("mul");
}
