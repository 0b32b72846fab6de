// MoNuSeg training-time augmentation on the GPU, reproducing the
// reference's PIL/torchvision pipeline byte for byte:
//   aug_monuseg_dataset.py:113-148 (_apply_joint_transforms): Image.resize BILINEAR
//   (image) / NEAREST (mask) -> hflip -> vflip -> rotate(angle, BILINEAR / NEAREST)
//   -> adjust_brightness -> adjust_contrast -> adjust_saturation -> adjust_hue ->
//   ToTensor.
// Every stage works on uint8 RGB (HWC) exactly like PIL's 8-bit images, with PIL's
// own arithmetic: the antialiasing resampler's 22-bit fixed-point coefficients
// (host-computed tables), the affine transform's double-precision coordinates and
// truncating bilinear filter, the 16.16 fixed-point nearest path for the mask,
// ImagingBlend's float32 blend with truncation, the L conversion
// (299/587/114 in 16-bit fixed point), and RGB<->HSV as in Convert.c.  Floating-point
// steps use explicit _rn intrinsics so no FMA contraction changes a rounding.
// The XML polygon rasterisation (monuseg_dataset.py:126-132, PIL ImageDraw.polygon) is
// Pillow's scan converter reproduced bit for bit (poly_edges_kernel / poly_scan_kernel).
#include <algorithm>

#include "common.h"

namespace ugpg {

constexpr int AA_PB = 22;  // PIL Resample.c PRECISION_BITS for 8-bit images

__device__ __forceinline__ uint8_t clip8_shift(int acc) {
    const int v = acc >> AA_PB;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// One separable pass of PIL's antialiasing resampler (ImagingResampleHorizontal_8bpc /
// Vertical_8bpc): out[.., o, ..] = clip8((2^21 + sum_t in[.., lo + t, ..] * k[o][t]) >> 22).
// `outer` rows of `inner` elements: horizontal pass = (B*H) x (W*C) with the tap stride
// C; vertical pass = B x (H*W*C) with the tap stride W*C.
__global__ void resample_aa_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                   int64_t outer, int n_in, int n_out, int inner_after,
                                   const int* __restrict__ bounds, const int* __restrict__ kk,
                                   int ksize) {
    // element (r, o, s): r = outer index, o = output position, s = position after the axis
    const int64_t total = outer * n_out * inner_after;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)(i % inner_after);
        const int64_t t = i / inner_after;
        const int o = (int)(t % n_out);
        const int64_t r = t / n_out;
        const int lo = bounds[2 * o], n = bounds[2 * o + 1];
        const uint8_t* src = in + (r * n_in + lo) * inner_after + s;
        const int* k = kk + (size_t)o * ksize;
        int acc = 1 << (AA_PB - 1);
        for (int x = 0; x < n; ++x) acc += (int)src[(int64_t)x * inner_after] * k[x];
        out[i] = clip8_shift(acc);
    }
}

// nearest resize with host-tabulated source indices (PIL ImagingScaleAffine)
__global__ void resize_nearest_u8_kernel(const uint8_t* __restrict__ in, int H, int W, int C,
                                         uint8_t* __restrict__ out, int OH, int OW, int64_t B,
                                         const int* __restrict__ ytab,
                                         const int* __restrict__ xtab) {
    const int64_t total = B * OH * OW * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        int64_t t = i / C;
        const int x = (int)(t % OW);
        t /= OW;
        const int y = (int)(t % OH);
        const int64_t b = t / OH;
        out[i] = in[((b * H + ytab[y]) * W + xtab[x]) * C + c];
    }
}

// per-sample geometric + brightness parameters (host-drawn, reference RNG order)
struct AugGeom {
    double a[6];      // affine source<-dest map of Image.rotate (PIL rounding applied)
    int fa[6];        // its 16.16 fixed-point form for the NEAREST mask path
    int rotate;       // 0 = no rotation (|angle| <= 1e-3, or angle % 360 == 0)
    int hflip, vflip;
    float brightness; // blend factor (1.0 = unchanged)
    int pad;
};

__device__ __forceinline__ uint8_t blend_u8(float in1, float in2, float alpha) {
    // ImagingBlend: float temp = in1 + alpha * (in2 - in1); clip; truncate
    const float t = __fadd_rn(in1, __fmul_rn(alpha, __fsub_rn(in2, in1)));
    if (t <= 0.f) return 0;
    if (t >= 255.f) return 255;
    return (uint8_t)(int)t;
}

__device__ __forceinline__ int lum8(int r, int g, int b) {
    return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16;  // PIL L24
}

// flips + rotation (image: bilinear_filter32RGB, mask: affine_fixed nearest) +
// brightness; accumulates the L sum of the result per sample (for contrast)
__global__ void augment_geom_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ msk,
                                    int S, int64_t B, const AugGeom* __restrict__ prm,
                                    uint8_t* __restrict__ oimg, uint8_t* __restrict__ omsk,
                                    unsigned* __restrict__ lsum) {
    const int64_t npix = (int64_t)S * S;
    const int64_t b = blockIdx.y;
    if (b >= B) return;
    const AugGeom p = prm[b];
    const uint8_t* im = img + b * npix * 3;
    const uint8_t* mk = msk + b * npix;
    unsigned part = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % S), y = (int)(i / S);
        // source pixel (sx, sy) of the flipped image = (fx(sx), fy(sy)) of the input
        auto fx = [&](int v) { return p.hflip ? S - 1 - v : v; };
        auto fy = [&](int v) { return p.vflip ? S - 1 - v : v; };
        uint8_t rgb[3] = {0, 0, 0};
        uint8_t mv = 0;
        if (!p.rotate) {
            const int64_t s = (int64_t)fy(y) * S + fx(x);
            rgb[0] = im[3 * s];
            rgb[1] = im[3 * s + 1];
            rgb[2] = im[3 * s + 2];
            mv = mk[s];
        } else {
            // affine_transform: xin = a0*(x+.5) + a1*(y+.5) + a2 (double, no contraction)
            const double xi = x + 0.5, yi = y + 0.5;
            double xin = __dadd_rn(__dadd_rn(__dmul_rn(p.a[0], xi), __dmul_rn(p.a[1], yi)), p.a[2]);
            double yin = __dadd_rn(__dadd_rn(__dmul_rn(p.a[3], xi), __dmul_rn(p.a[4], yi)), p.a[5]);
            if (xin >= 0.0 && xin < S && yin >= 0.0 && yin < S) {
                xin = __dsub_rn(xin, 0.5);
                yin = __dsub_rn(yin, 0.5);
                const int xf = (int)floor(xin), yf = (int)floor(yin);
                const double dx = __dsub_rn(xin, (double)xf), dy = __dsub_rn(yin, (double)yf);
                const int x0 = min(max(xf, 0), S - 1), x1 = min(max(xf + 1, 0), S - 1);
                const int y0 = min(max(yf, 0), S - 1);
                const bool has1 = yf + 1 >= 0 && yf + 1 < S;
                const int y1 = has1 ? yf + 1 : y0;
                const int64_t r0 = (int64_t)fy(y0) * S, r1 = (int64_t)fy(y1) * S;
                const int64_t c0 = fx(x0), c1 = fx(x1);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double a0 = im[3 * (r0 + c0) + c], b0 = im[3 * (r0 + c1) + c];
                    const double v1 = __dadd_rn(a0, __dmul_rn(__dsub_rn(b0, a0), dx));
                    double v2 = v1;
                    if (has1) {
                        const double a1 = im[3 * (r1 + c0) + c], b1 = im[3 * (r1 + c1) + c];
                        v2 = __dadd_rn(a1, __dmul_rn(__dsub_rn(b1, a1), dx));
                    }
                    const double v = __dadd_rn(v1, __dmul_rn(__dsub_rn(v2, v1), dy));
                    rgb[c] = (uint8_t)(v <= 0.0 ? 0 : (v >= 255.0 ? 255 : (int)v));
                }
            }
            // affine_fixed (16.16): xx = xo + y*a1 + x*a0, source = xx >> 16
            const int xx = p.fa[2] + y * p.fa[1] + x * p.fa[0];
            const int yy = p.fa[5] + y * p.fa[4] + x * p.fa[3];
            const int sx = xx >> 16, sy = yy >> 16;
            if (sx >= 0 && sx < S && sy >= 0 && sy < S) mv = mk[(int64_t)fy(sy) * S + fx(sx)];
        }
        if (p.brightness != 1.f) {
#pragma unroll
            for (int c = 0; c < 3; ++c) rgb[c] = blend_u8(0.f, (float)rgb[c], p.brightness);
        }
        uint8_t* o = oimg + (b * npix + i) * 3;
        o[0] = rgb[0];
        o[1] = rgb[1];
        o[2] = rgb[2];
        omsk[b * npix + i] = mv;
        part += (unsigned)lum8(rgb[0], rgb[1], rgb[2]);
    }
    // per-sample L sum (integer atomics: exact and order-independent)
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if ((threadIdx.x & 63) == 0 && part) atomicAdd(lsum + b, part);
}

struct AugColor {
    int jitter;      // 0 = no colour stage
    float contrast, saturation;
    int hue_shift;   // uint8 added to H (mod 256)
};

// PIL Convert.c rgb2hsv_row (float/double mix reproduced)
__device__ __forceinline__ void rgb2hsv_pil(int r, int g, int b, int& uh, int& us, int& uv) {
    const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
    uv = maxc;
    if (minc == maxc) {
        uh = 0;
        us = 0;
        return;
    }
    const float cr = (float)(maxc - minc);
    const float s = __fdiv_rn(cr, (float)maxc);
    const float rc = __fdiv_rn((float)(maxc - r), cr);
    const float gc = __fdiv_rn((float)(maxc - g), cr);
    const float bc = __fdiv_rn((float)(maxc - b), cr);
    float h;
    if (r == maxc) h = __fsub_rn(bc, gc);
    else if (g == maxc) h = (float)__dsub_rn(__dadd_rn(2.0, (double)rc), (double)bc);
    else h = (float)__dsub_rn(__dadd_rn(4.0, (double)gc), (double)rc);
    h = (float)fmod(__dadd_rn(__ddiv_rn((double)h, 6.0), 1.0), 1.0);
    const int ih = (int)__dmul_rn((double)h, 255.0), is = (int)__dmul_rn((double)s, 255.0);
    uh = ih < 0 ? 0 : (ih > 255 ? 255 : ih);
    us = is < 0 ? 0 : (is > 255 ? 255 : is);
}

__device__ __forceinline__ int round_pos(double v) { return (int)floor(__dadd_rn(v, 0.5)); }

// PIL Convert.c hsv2rgb_row
__device__ __forceinline__ void hsv2rgb_pil(int h, int s, int v, int& r, int& g, int& b) {
    if (s == 0) {
        r = g = b = v;
        return;
    }
    const double h6 = __ddiv_rn(__dmul_rn((double)(float)h, 6.0), 255.0);
    const int i = (int)floor(h6);
    const float f = (float)__dsub_rn(h6, (double)(float)i);
    const float fs = (float)__ddiv_rn((double)(float)s, 255.0);
    const double vf = (double)(float)v;
    int p = round_pos(__dmul_rn(vf, __dsub_rn(1.0, (double)fs)));
    int q = round_pos(__dmul_rn(vf, __dsub_rn(1.0, (double)__fmul_rn(fs, f))));
    int t = round_pos(__dmul_rn(vf, __dsub_rn(1.0, __dmul_rn((double)fs, __dsub_rn(1.0, (double)f)))));
    p = min(max(p, 0), 255);
    q = min(max(q, 0), 255);
    t = min(max(t, 0), 255);
    switch (i % 6) {
        case 0: r = v, g = t, b = p; break;
        case 1: r = q, g = v, b = p; break;
        case 2: r = p, g = v, b = t; break;
        case 3: r = p, g = q, b = v; break;
        case 4: r = t, g = p, b = v; break;
        default: r = v, g = p, b = q; break;
    }
}

// contrast -> saturation -> hue -> ToTensor (NCHW float through the exact /255 table);
// mask -> float
__global__ void augment_color_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ msk,
                                     int S, int64_t B, const AugColor* __restrict__ prm,
                                     const unsigned* __restrict__ lsum,
                                     const float* __restrict__ u8_to_f32,
                                     float* __restrict__ out, float* __restrict__ omask) {
    const int64_t npix = (int64_t)S * S;
    const int64_t b = blockIdx.y;
    if (b >= B) return;
    const AugColor p = prm[b];
    // ImageStat mean of L = sum / count (double); degenerate grey level int(mean + 0.5)
    const int mean = (int)__dadd_rn(__ddiv_rn((double)lsum[b], (double)npix), 0.5);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* q = img + (b * npix + i) * 3;
        int r = q[0], g = q[1], bl = q[2];
        if (p.jitter) {
            if (p.contrast != 1.f) {
                r = blend_u8((float)mean, (float)r, p.contrast);
                g = blend_u8((float)mean, (float)g, p.contrast);
                bl = blend_u8((float)mean, (float)bl, p.contrast);
            }
            if (p.saturation != 1.f) {
                const float l = (float)lum8(r, g, bl);
                r = blend_u8(l, (float)r, p.saturation);
                g = blend_u8(l, (float)g, p.saturation);
                bl = blend_u8(l, (float)bl, p.saturation);
            }
            {  // adjust_hue: the HSV round trip runs even for a zero shift (it is lossy)
                int h, s, v;
                rgb2hsv_pil(r, g, bl, h, s, v);
                h = (h + p.hue_shift) & 255;
                hsv2rgb_pil(h, s, v, r, g, bl);
            }
        }
        float* o = out + b * 3 * npix + i;
        o[0] = u8_to_f32[r];
        o[npix] = u8_to_f32[g];
        o[2 * npix] = u8_to_f32[bl];
        omask[b * npix + i] = (float)msk[b * npix + i];
    }
}

// ---------------------------------------------------------------------------
// Filled polygons, Pillow 12's scan converter (libImaging/Draw.c ImagingDrawPolygon +
// polygon_generic + hline8; restated and pinned in oracle/polygon_ref.py, whose header
// lists the rules).  Float steps in float without contraction,
// the negative-argument rounding macros in double, as Pillow's x86 build evaluates them.
// (tests/test_asm_audit.py checks the scan kernel holds no fused multiply-add)
struct PolyEdge {
    int x0, y0, xmin, ymin, xmax, ymax;
    float dx;
    int pad;
};
struct PolyInfo {
    int nedges, ymin, ymax, pad;
};

// C (int) of a double on x86: toward zero, out of range -> INT_MIN
__device__ __forceinline__ int trunc_int_x86(double v) {
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : (int)0x80000000u;
}
__device__ __forceinline__ void poly_hline(uint8_t* mask, int H, int W, int x0, int y, int x1,
                                           uint8_t ink) {
    if (y < 0 || y >= H) return;
    if (x0 < 0) {
        if (x1 < 0) return;
        x0 = 0;
    } else if (x0 >= W || x1 < 0) {
        return;
    }
    if (x1 >= W) x1 = W - 1;
    uint8_t* row = mask + (size_t)y * W;
    for (int x = x0; x <= x1; ++x) row[x] = ink;
}
__device__ __forceinline__ float poly_x_at(const PolyEdge& e, int y) {
    // separately rounded product and sum: contraction off here (HIP's __fmul_rn and
    // __fadd_rn are plain operators, which -O3 fuses into one v_fma_f32)
#pragma clang fp contract(off)
    const float m = (float)(y - e.y0) * e.dx;
    return m + (float)e.x0;
}
__device__ __forceinline__ int poly_round_up(float f) {
    if (f >= 0.f) return (int)floorf(__fadd_rn(f, 0.5f));
    return -(int)floor(__dadd_rn(fabs((double)f), 0.5));
}
__device__ __forceinline__ int poly_round_down(float f) {
    if (f >= 0.f) return (int)ceilf(__fsub_rn(f, 0.5f));
    return -(int)ceil(__dsub_rn(fabs((double)f), 0.5));
}

// one thread per polygon: vertices -> edges (in order; consecutive horizontal edges in the
// same direction merged), horizontal edges drawn as spans, the row range recorded
__global__ void poly_edges_kernel(const double* __restrict__ xy, const int64_t* __restrict__ off,
                                  int64_t npoly, PolyEdge* __restrict__ edges,
                                  PolyInfo* __restrict__ info, uint8_t* mask, int H, int W,
                                  uint8_t ink) {
    const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (p >= npoly) return;
    const int64_t v0 = off[p];
    const int count = (int)(off[p + 1] - v0);
    if (count < 2) {  // (the host refuses these; PIL raises) -- no rows
        info[p] = PolyInfo{0, 1, 0, 0};
        return;
    }
    PolyEdge* e = edges + v0;
    auto X = [&](int i) { return trunc_int_x86(xy[2 * (v0 + i)]); };
    auto Y = [&](int i) { return trunc_int_x86(xy[2 * (v0 + i) + 1]); };
    auto add = [&](int n, int x0, int y0, int x1, int y1) {
        PolyEdge q;
        q.xmin = x0 <= x1 ? x0 : x1;
        q.xmax = x0 <= x1 ? x1 : x0;
        q.ymin = y0 <= y1 ? y0 : y1;
        q.ymax = y0 <= y1 ? y1 : y0;
        q.dx = y0 == y1 ? 0.f : __fdiv_rn((float)(x1 - x0), (float)(y1 - y0));
        q.x0 = x0;
        q.y0 = y0;
        q.pad = 0;
        e[n] = q;
    };
    int n = 0, i = 0;
    for (i = 0; i < count - 1; ++i) {
        const int x0 = X(i), y0 = Y(i), x1 = X(i + 1), y1 = Y(i + 1);
        if (y0 == y1 && i != 0 && y0 == Y(i - 1)) {
            const int xp = X(i - 1);
            if (x1 > x0 && x0 > xp) {
                e[n - 1].xmax = x1;
                continue;
            }
            if (x1 < x0 && x0 < xp) {
                e[n - 1].xmin = x1;
                continue;
            }
        }
        add(n++, x0, y0, x1, y1);
    }
    if (X(i) != X(0) || Y(i) != Y(0)) add(n++, X(i), Y(i), X(0), Y(0));
    // the row range over every edge; horizontal edges are drawn here and dropped from the
    // table (compacted in place, order kept)
    int ymin = H - 1, ymax = 0, m = 0;
    for (int k = 0; k < n; ++k) {
        const PolyEdge q = e[k];
        ymin = min(ymin, q.ymin);
        ymax = max(ymax, q.ymax);
        if (q.ymin == q.ymax) {
            poly_hline(mask, H, W, q.xmin, q.ymin, q.xmax, ink);
            continue;
        }
        e[m++] = q;
    }
    info[p] = PolyInfo{m, max(ymin, 0), min(ymax, H), 0};
}

// one 64-lane workgroup per polygon, a row per lane: the row's edge crossings (with the
// corner rule), sorted, filled pairwise; lane scratch = 2 * (vertex count) floats
__global__ void __launch_bounds__(64) poly_scan_kernel(const int64_t* __restrict__ off,
                                                       const PolyEdge* __restrict__ edges,
                                                       const PolyInfo* __restrict__ info,
                                                       float* __restrict__ scratch, uint8_t* mask,
                                                       int H, int W, uint8_t ink) {
    const int64_t p = blockIdx.x;
    const int64_t v0 = off[p];
    const int cap = 2 * (int)(off[p + 1] - v0);
    const PolyInfo pi = info[p];
    const PolyEdge* e = edges + v0;
    float* xx = scratch + 128 * v0 + (int64_t)threadIdx.x * cap;
    for (int y = pi.ymin + (int)threadIdx.x; y <= pi.ymax; y += 64) {
        int j = 0;
        for (int i = 0; i < pi.nedges; ++i) {
            const PolyEdge cur = e[i];
            if (y < cur.ymin || y > cur.ymax) continue;
            float x = poly_x_at(cur, y);
            if (y == cur.ymax && y < pi.ymax) {
                xx[j++] = x;
                xx[j++] = x;
                continue;
            }
            if ((y == cur.ymin || y == cur.ymax) && cur.dx != 0.f) {
                const int adj = y == cur.ymax ? y - 1 : y + 1;
                for (int k = 0; k < i; ++k) {
                    const PolyEdge o = e[k];
                    if (!((y == o.ymin || y == o.ymax) && o.dx != 0.f)) continue;
                    if (roundf(x) != roundf(poly_x_at(o, y))) continue;
                    if (adj < o.ymin || adj > o.ymax) continue;
                    const float ac = poly_x_at(cur, adj), ao = poly_x_at(o, adj);
                    if (x > __fadd_rn(ac, 1.f) && x > __fadd_rn(ao, 1.f))
                        x = __fadd_rn(roundf(fmaxf(ac, ao)), 1.f);
                    else if (x < __fsub_rn(ac, 1.f) && x < __fsub_rn(ao, 1.f))
                        x = __fsub_rn(roundf(fminf(ac, ao)), 1.f);
                    break;
                }
            }
            xx[j++] = x;
        }
        for (int a = 1; a < j; ++a) {  // insertion sort (a handful of crossings per row)
            const float v = xx[a];
            int b = a - 1;
            while (b >= 0 && xx[b] > v) {
                xx[b + 1] = xx[b];
                --b;
            }
            xx[b + 1] = v;
        }
        for (int a = 1; a < j; a += 2)
            poly_hline(mask, H, W, poly_round_up(xx[a - 1]), y, poly_round_down(xx[a]), ink);
    }
}

}  // namespace ugpg

using namespace ugpg;

extern "C" int ugpg_resample_aa_u8(const uint8_t* in, int64_t outer, int n_in, int n_out,
                                   int inner_after, const int* bounds, const int* kk, int ksize,
                                   uint8_t* out, void* stream) {
    if (!in || !out || !bounds || !kk || outer <= 0 || n_in <= 0 || n_out <= 0 ||
        inner_after <= 0 || ksize <= 0) {
        set_error("resample_aa_u8: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(resample_aa_kernel, dim3(stream_grid(outer * n_out * inner_after)),
                       dim3(256), 0, as_stream(stream), in, out, outer, n_in, n_out, inner_after,
                       bounds, kk, ksize);
    return check_launch("resample_aa_u8");
}

extern "C" int ugpg_resize_nearest_u8(const uint8_t* in, int64_t B, int H, int W, int C,
                                      const int* ytab, const int* xtab, uint8_t* out, int OH,
                                      int OW, void* stream) {
    if (!in || !out || !ytab || !xtab || B <= 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 ||
        OW <= 0) {
        set_error("resize_nearest_u8: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(resize_nearest_u8_kernel, dim3(stream_grid(B * OH * OW * C)), dim3(256), 0,
                       as_stream(stream), in, H, W, C, out, OH, OW, B, ytab, xtab);
    return check_launch("resize_nearest_u8");
}

// struct sizes of the per-sample parameter records (host layout check)
extern "C" int ugpg_augment_param_sizes(int* geom, int* color) {
    if (!geom || !color) return UGPG_ERR_INVALID;
    *geom = (int)sizeof(AugGeom);
    *color = (int)sizeof(AugColor);
    return UGPG_OK;
}

extern "C" int ugpg_augment_geom(const uint8_t* img, const uint8_t* mask, int S, int64_t B,
                                 const void* params, uint8_t* out_img, uint8_t* out_mask,
                                 unsigned* lsum, void* stream) {
    if (!img || !mask || !params || !out_img || !out_mask || !lsum || S <= 0 || B <= 0 ||
        B > 65535 || (int64_t)S * S > (1ll << 24)) {
        set_error("augment_geom: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(lsum, 0, B * sizeof(unsigned), st) != hipSuccess) {
        set_error("augment_geom: memset failed");
        return UGPG_ERR_LAUNCH;
    }
    const unsigned gx = (unsigned)std::min<int64_t>(cdiv((int64_t)S * S, 256), 256);
    hipLaunchKernelGGL(augment_geom_kernel, dim3(gx, (unsigned)B), dim3(256), 0, st, img, mask, S,
                       B, static_cast<const AugGeom*>(params), out_img, out_mask, lsum);
    return check_launch("augment_geom");
}

extern "C" int ugpg_augment_color(const uint8_t* img, const uint8_t* mask, int S, int64_t B,
                                  const void* params, const unsigned* lsum,
                                  const float* u8_to_f32, float* out, float* out_mask,
                                  void* stream) {
    if (!img || !mask || !params || !lsum || !u8_to_f32 || !out || !out_mask || S <= 0 ||
        B <= 0 || B > 65535) {
        set_error("augment_color: bad arguments");
        return UGPG_ERR_INVALID;
    }
    const unsigned gx = (unsigned)std::min<int64_t>(cdiv((int64_t)S * S, 256), 256);
    hipLaunchKernelGGL(augment_color_kernel, dim3(gx, (unsigned)B), dim3(256), 0,
                       as_stream(stream), img, mask, S, B, static_cast<const AugColor*>(params),
                       lsum, u8_to_f32, out, out_mask);
    return check_launch("augment_color");
}

extern "C" size_t ugpg_rasterize_polygons_ws_size(int64_t nverts, int64_t npoly) {
    if (nverts < 0 || npoly < 0) return 0;
    // edges (<= vertices), per-polygon info, per-lane crossing scratch (64 lanes x 2 x n)
    return (size_t)nverts * sizeof(PolyEdge) + (size_t)npoly * sizeof(PolyInfo) +
           (size_t)nverts * 128 * sizeof(float);
}

extern "C" int ugpg_rasterize_polygons(const double* xy, const int64_t* off, int64_t npoly,
                                       int64_t nverts, uint8_t* mask, int H, int W, int ink,
                                       void* ws, size_t ws_bytes, void* stream) {
    if (!xy || !off || !mask || !ws || npoly <= 0 || nverts < 2 * npoly || H <= 0 || W <= 0 ||
        ink < 0 || ink > 255 || npoly > (1ll << 31) - 1) {
        set_error("rasterize_polygons: bad arguments");
        return UGPG_ERR_INVALID;
    }
    if (ws_bytes < ugpg_rasterize_polygons_ws_size(nverts, npoly)) {
        set_error("rasterize_polygons: workspace too small");
        return UGPG_ERR_WORKSPACE;
    }
    hipStream_t st = as_stream(stream);
    PolyEdge* edges = static_cast<PolyEdge*>(ws);
    PolyInfo* info = reinterpret_cast<PolyInfo*>(edges + nverts);
    float* scratch = reinterpret_cast<float*>(info + npoly);
    hipLaunchKernelGGL(poly_edges_kernel, dim3((unsigned)cdiv(npoly, 64)), dim3(64), 0, st, xy, off,
                       npoly, edges, info, mask, H, W, (uint8_t)ink);
    if (int r = check_launch("rasterize_polygons(edges)")) return r;
    hipLaunchKernelGGL(poly_scan_kernel, dim3((unsigned)npoly), dim3(64), 0, st, off, edges, info,
                       scratch, mask, H, W, (uint8_t)ink);
    return check_launch("rasterize_polygons(scan)");
}
