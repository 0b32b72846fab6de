// Shared pieces of the 3x3 convolution kernels (conv.hip: fp32 MFMA path,
// conv_x6.hip: split-bf16 path): launch arguments, the output-pixel map of an
// MFMA row, and the common epilogue (bias, dual-destination store, per-tile
// BatchNorm partials).
#pragma once
#include "common.h"

namespace ugpg {

struct ConvFwdArgs {
    const float* src0;
    const float* sc0;
    const float* sh0;
    int C0;
    const float* src1;
    const float* sc1;
    const float* sh1;
    int C1;
    const void* wpk;
    const float* bias;
    float* out0;
    float* out1;
    int split, acc0, acc1;
    float* stats;
    int B, H, W, Cin, Cout;
    int tiles_x, tiles_y, ntiles;
    // BatchNorm-backward partials of out0 (ugpg_conv_t.bnb_*; bnb_part == nullptr: off)
    YRef bnb_y;
    const float* bnb_mean;
    const float* bnb_invstd;
    const float* bnb_scale;
    const float* bnb_shift;
    float* bnb_part;
    // bf16 activations (ugpg_src_t.data_bf16, ugpg_conv_t.out_bf16): read by / written by
    // the single-piece persistent form; nullptr: none.  out0 == nullptr with out0_16 set:
    // the output is stored in bf16 only (stats and partials of the rounded values)
    const __bf16* src0_16;
    const __bf16* src1_16;
    __bf16* out0_16;
};

// Output pixel (row*TW + col inside the tile) of GEMM row m.  PERM16 is the
// 16-wide tile map of the split-bf16 kernel: each 32-row MFMA tile covers two
// image rows and its rows are permuted so that every 16-lane ds_read_b128 group
// touches 8 pixels of each of the two halo rows (conflict-free with a 24-pixel
// halo row pitch).  Rows are permuted in aligned blocks of 4.
template <int TW, bool PERM16>
__device__ __forceinline__ int tile_pixel(int m) {
    if constexpr (PERM16) {
        const int i = m & 31;
        // block b = i>>2 -> first pixel / 4: {0, 2, 3, 1, 6, 4, 5, 7}
        constexpr unsigned P = 0u | (2u << 3) | (3u << 6) | (1u << 9) | (6u << 12) | (4u << 15) |
                               (5u << 18) | (7u << 21);
        return (m >> 5) * 32 + 4 * ((P >> (3 * (i >> 2))) & 7u) + (i & 3);
    } else {
        return m;
    }
}

// acc[mt][nt]: the 32x32 fp32 tile (mt, nt) of wave (wm, wn) in the standard
// 32x32 C/D map (row (r&3)+8(r>>2)+4h, column lane&31).
template <int TH, int TW, int BN, int WM, int WN, int MT, int NT, bool PERM16>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs& a, f32x16 (&acc)[MT][NT],
                                              float* smem, int tile, int b, int ty0, int tx0,
                                              int n0, int wm, int wn) {
    constexpr int WTM = MT * 32, WTN = NT * 32;
    const int tid = threadIdx.x, lane = tid & 63;
    const int vh = min(TH, a.H - ty0), vw = min(TW, a.W - tx0);
    float* out;
    int ostride, ocol0, oacc;
    if (n0 < a.split) {
        out = a.out0;
        ostride = a.split;
        ocol0 = n0;
        oacc = a.acc0;
    } else {
        out = a.out1;
        ostride = a.Cout - a.split;
        ocol0 = n0 - a.split;
        oacc = a.acc1;
    }
    float psum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int nl = wn * WTN + nt * 32 + (lane & 31);
        const float bv = a.bias ? a.bias[n0 + nl] : 0.f;
        psum[nt] = 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = tile_pixel<TW, PERM16>(wm * WTM + mt * 32 + (r & 3) + 8 * (r >> 2) +
                                                     4 * (lane >> 5));
                const int py = m / TW, px = m % TW;
                const float v = acc[mt][nt][r] + bv;
                acc[mt][nt][r] = v;
                if (py < vh && px < vw) {
                    const size_t o =
                        ((size_t)(b * a.H + ty0 + py) * a.W + tx0 + px) * ostride + ocol0 + nl;
                    out[o] = oacc ? out[o] + v : v;
                    psum[nt] += v;
                }
            }
    }
    if (a.stats == nullptr) return;
    float* red = smem;            // [WM][BN]
    float* tot = smem + WM * BN;  // [BN]
    const float cnt = (float)(vh * vw);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const float s = psum[nt] + __shfl_xor(psum[nt], 32, 64);
        if (lane < 32) red[wm * BN + wn * WTN + nt * 32 + lane] = s;
    }
    __syncthreads();
    if (tid < BN) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) s += red[w * BN + tid];
        tot[tid] = s;
    }
    __syncthreads();
    float pq[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int nl = wn * WTN + nt * 32 + (lane & 31);
        const float mu = tot[nl] / cnt;
        float q = 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = tile_pixel<TW, PERM16>(wm * WTM + mt * 32 + (r & 3) + 8 * (r >> 2) +
                                                     4 * (lane >> 5));
                if (m / TW < vh && m % TW < vw) {
                    const float d = acc[mt][nt][r] - mu;
                    q = fmaf(d, d, q);
                }
            }
        pq[nt] = q + __shfl_xor(q, 32, 64);
    }
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
        if (lane < 32) red[wm * BN + wn * WTN + nt * 32 + lane] = pq[nt];
    __syncthreads();
    if (tid < BN) {
        float q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) q += red[w * BN + tid];
        const size_t n = n0 + tid, T = a.ntiles;
        a.stats[(0 * (size_t)a.Cout + n) * T + tile] = cnt;
        a.stats[(1 * (size_t)a.Cout + n) * T + tile] = tot[tid];
        a.stats[(2 * (size_t)a.Cout + n) * T + tile] = q;
    }
}

struct WgradArgs {
    const float* src0;
    const float* sc0;
    const float* sh0;
    int C0;
    const float* src1;
    const float* sc1;
    const float* sh1;
    int C1;
    const float* dy;
    // bf16 activation storage (src0/src1 == nullptr; the x6w single-piece form only)
    const __bf16* src0_16;
    const __bf16* src1_16;
    // dy stored in bf16 (dy == nullptr; the x6w single-piece form only)
    const __bf16* dy16;
    // dy formed while loading from the following BatchNorm(+ReLU) backward (ugpg_bn_lazy_t;
    // bn_da == nullptr: off; the split-bf16 x6w form): bn_dy_out receives it (nullable)
    const float* bn_da;
    const float* bn_y;
    const float* bn_mean;
    const float* bn_invstd;
    const float* bn_scale;
    const float* bn_shift;
    const float* bn_coef;
    float* bn_dy_out;
    const float* bn_rsrc;    // MaxPool2d route of da (nullable): pooled gradient, argmax
    const uint8_t* bn_ram;
    const __bf16* bn_y16;    // y stored in bf16 (bn_y == nullptr; the image layer's kernel only)
    int Cout, Cin;
    float* part;
    float* dbpart;
    int B, H, W;
    int tiles_x, tiles_y, ntiles, nsplit, tps;
};

// split-bf16 path (conv_x6.hip)
// np: bf16 pieces (3 or 1); returns which of the optional outputs the launched form wrote
// itself: FWD_WROTE_BNB (a.bnb_part), FWD_WROTE_OUT16 (a.out0_16)
constexpr int FWD_WROTE_BNB = 1, FWD_WROTE_OUT16 = 2;
int launch_fwd_x6(const ConvFwdArgs& a, int np, hipStream_t st);
// the image layer's direct fp32 forward (conv_x6.hip): shape predicate,
// BatchNorm slot count (nwm row groups per 8 x 32 tile), launch (false: not applicable)
bool img_fwd_eligible(int W, int C0, int C1, int Cout);
int img_fwd_slots(int B, int H, int W, int nwm);
bool launch_img_fwd(const ConvFwdArgs& a, bool wf32, hipStream_t st);  // writes out0_16 too
// bn.hip: the per-slot BatchNorm-backward reduction (partials layout of ugpg_conv_t.bnb_part)
void launch_bn_bwd_reduce(const float* da, YRef y, int64_t npix, int C, const float* mean,
                          const float* invstd, const float* scale, const float* shift, float* part,
                          int nslots, hipStream_t st);
// batched weight packing (ugpg_pack_conv3x3_batch), kernel-argument descriptors
struct PackItem {
    const float* w;
    void* wpk;
    int Cout, Cin, Cin_pad, mode;
};
constexpr int PACK_BATCH_MAX = 48;
struct PackBatch {
    PackItem item[PACK_BATCH_MAX];
    int first[PACK_BATCH_MAX + 1];
    int n;
};
void launch_pack_x6_batch(const PackItem* items, int n, int np, hipStream_t st);
// the split-bf16 / bf16 forward form of a shape (np = bf16 pieces: 3 split, 1 bf16; N =
// output channels): pixel tile th x tw, 64-column weight slabs per item, pixel groups
// (BatchNorm partial slots) per tile, persistent kernel or the single-stage one
struct X6Form {
    int th, tw, nslab, wm;
    bool persistent;
};
X6Form x6_fwd_form(int B, int H, int W, int K, int N, int np);  // K: input channels
int fwd_x6_stat_slots(const X6Form& f, int B, int H, int W);  // BatchNorm partial slots written
void launch_wgrad_x6(const WgradArgs& a, int np, hipStream_t st);
// split plan of the persistent split-bf16 wgrad (deterministic: planned for `cus` CUs)
void wgrad_x6w_plan(int ntiles, int Cout, int Cin, int cus, int& nsplit, int& tps);
constexpr int WGX6_TW = 16, WGX6W_TH = 4;  // pixel tile (4 x 16) of the split-bf16 wgrad
void launch_pack_x6(const float* w, void* wpk, int Cout, int Cin, int Cin_pad, int mode, int np,
                    hipStream_t st);

}  // namespace ugpg
