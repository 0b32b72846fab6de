// Classification-head kernels for the Herlev configuration (BASELINE config 4):
//   dropout masks   (nn.Dropout in the classifier, Herlev/train_herlev.py:66-77)
//   UG cross-entropy (uncertainty_guided_forward_pass, train_herlev.py:216-296)
//   Adam            (setup_optimizer_scheduler, train_herlev.py:178-194)
// The batch here is tiny (B x K = 16 x 7), so the loss kernels run as one block;
// they exist so that the whole step stays on the device without host syncs.
#include "common.h"

namespace ugpg {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void dropout_mask_kernel(float* mask, int64_t n, float p, uint64_t seed) {
    const float keep = 1.0f / (1.0f - p);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float u = (float)(mix64(seed ^ mix64((uint64_t)i)) >> 40) * (1.0f / 16777216.0f);
        mask[i] = u >= p ? keep : 0.0f;
    }
}

// One block.  ce_b = logsumexp(x_b) - x_b[y_b]; u_b = H(softmax(prev_b))/log K
__global__ void __launch_bounds__(256) ce_ug_fwd_kernel(const float* x, const int64_t* y,
                                                        const float* prev, const float* cw, int B,
                                                        int K, float alpha, float* out,
                                                        float* wts) {
    __shared__ double s_ce[256], s_w[256], s_cw[256], s_wce[256], s_ok[256];
    double ce_acc = 0, wsum = 0, cwsum = 0, wce = 0, ok = 0;
    for (int b = threadIdx.x; b < B; b += 256) {
        const float* xb = x + (size_t)b * K;
        float m = -INFINITY;
        int am = 0;
        for (int k = 0; k < K; ++k)
            if (xb[k] > m) {  // first maximum, as torch.argmax
                m = xb[k];
                am = k;
            }
        double se = 0;
        for (int k = 0; k < K; ++k) se += exp((double)(xb[k] - m));
        const int yb = (int)y[b];
        const double ce = (double)m + log(se) - (double)xb[yb];
        ok += (am == yb) ? 1.0 : 0.0;
        double w = 1.0;
        if (prev) {
            const float* pb = prev + (size_t)b * K;
            float mp = -INFINITY;
            for (int k = 0; k < K; ++k) mp = fmaxf(mp, pb[k]);
            float sp = 0.f;
            for (int k = 0; k < K; ++k) sp += expf(pb[k] - mp);
            float h = 0.f;
            for (int k = 0; k < K; ++k) {
                const float pk = expf(pb[k] - mp) / sp;
                h -= pk * logf(pk + 1e-8f);
            }
            w = 1.0 + (double)alpha * (double)(h / logf((float)K));
        }
        if (wts) wts[b] = (float)w;
        const double cwy = cw ? (double)cw[yb] : 1.0;
        ce_acc += cwy * ce;   // class-weighted CE numerator (base loss)
        cwsum += cwy;
        wce += w * ce;        // sample-weighted CE (final loss)
        wsum += w;
    }
    s_ce[threadIdx.x] = ce_acc;
    s_cw[threadIdx.x] = cwsum;
    s_wce[threadIdx.x] = wce;
    s_w[threadIdx.x] = wsum;
    s_ok[threadIdx.x] = ok;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            s_ce[threadIdx.x] += s_ce[threadIdx.x + s];
            s_cw[threadIdx.x] += s_cw[threadIdx.x + s];
            s_wce[threadIdx.x] += s_wce[threadIdx.x + s];
            s_w[threadIdx.x] += s_w[threadIdx.x + s];
            s_ok[threadIdx.x] += s_ok[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[4] = (float)s_ok[0];
        const double base = s_ce[0] / s_cw[0];
        out[1] = (float)base;
        out[0] = prev ? (float)(s_wce[0] / B) : (float)base;
        const double mw = s_w[0] / B;
        double q = 0;
        if (wts)
            for (int b = 0; b < B; ++b) q += ((double)wts[b] - mw) * ((double)wts[b] - mw);
        out[2] = prev ? (float)mw : 0.f;
        out[3] = prev ? (float)(B > 1 ? sqrt(q / (B - 1)) : NAN) : 0.f;
    }
}

// d final / d x.  With prev: w_b/B (softmax - onehot); else class-weighted mean CE.
__global__ void ce_ug_bwd_kernel(const float* x, const int64_t* y, const float* wts,
                                 const float* cw, int B, int K, const float* gout, float* dx) {
    __shared__ float norm;
    if (threadIdx.x == 0) {
        float s = 0.f;
        if (!wts)
            for (int b = 0; b < B; ++b) s += cw ? cw[(int)y[b]] : 1.0f;
        norm = wts ? (float)B : s;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        const float* xb = x + (size_t)b * K;
        float m = -INFINITY;
        for (int k = 0; k < K; ++k) m = fmaxf(m, xb[k]);
        float se = 0.f;
        for (int k = 0; k < K; ++k) se += expf(xb[k] - m);
        const int yb = (int)y[b];
        const float w = wts ? wts[b] : (cw ? cw[yb] : 1.0f);
        const float g = gout[0] * w / norm;
        for (int k = 0; k < K; ++k) {
            const float p = expf(xb[k] - m) / se;
            dx[(size_t)b * K + k] = g * (p - (k == yb ? 1.0f : 0.0f));
        }
    }
}

__global__ void adam_kernel(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                            float b1, float b2, float eps, float wd, float bc1, float bc2s,
                            float gs) {
    const float step_size = lr / bc1;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float pv = p[i];
        float gv = g[i];
        if (gs != 1.0f) gv *= gs;
        if (wd != 0.0f) gv = gv + wd * pv;
        const float mv = m[i] + (gv - m[i]) * (1.0f - b1);   // torch: lerp_(grad, 1-beta1)
        const float vv = v[i] * b2 + (1.0f - b2) * (gv * gv);
        m[i] = mv;
        v[i] = vv;
        const float denom = sqrtf(vv) / bc2s + eps;
        p[i] = pv + (-step_size) * (mv / denom);
    }
}

}  // namespace ugpg

using namespace ugpg;

extern "C" int ugpg_dropout_mask(float* mask, int64_t n, float p, uint64_t seed, void* stream) {
    if (!mask || n < 0 || p < 0.f || p >= 1.f) {
        set_error("dropout_mask: bad arguments (p=%f)", p);
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream),
                       mask, n, p, seed);
    return check_launch("dropout_mask");
}

extern "C" int ugpg_ce_ug_fwd(const float* x, const int64_t* y, const float* prev,
                              const float* class_weights, int B, int K, float alpha, float* out,
                              float* weights, void* stream) {
    if (!x || !y || !out || B <= 0 || K <= 2 || (prev && !weights)) {
        set_error("ce_ug_fwd: bad arguments (B=%d K=%d; binary heads are not supported)", B, K);
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(ce_ug_fwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), x, y, prev,
                       class_weights, B, K, alpha, out, weights);
    return check_launch("ce_ug_fwd");
}

extern "C" int ugpg_ce_ug_bwd(const float* x, const int64_t* y, const float* weights,
                              const float* class_weights, int B, int K, const float* gout,
                              float* dx, void* stream) {
    if (!x || !y || !gout || !dx || B <= 0 || K <= 0) {
        set_error("ce_ug_bwd: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(ce_ug_bwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), x, y, weights,
                       class_weights, B, K, gout, dx);
    return check_launch("ce_ug_bwd");
}

extern "C" int ugpg_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                              float beta1, float beta2, float eps, float weight_decay, int64_t step,
                              float grad_scale, void* stream) {
    if (!p || !g || !m || !v || step < 1) {
        set_error("adam_step: bad arguments");
        return UGPG_ERR_INVALID;
    }
    if (n == 0) return UGPG_OK;
    const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
    const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
    hipLaunchKernelGGL(adam_kernel, dim3(stream_grid(n)), dim3(256), 0, as_stream(stream), p, g, m,
                       v, n, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, grad_scale);
    return check_launch("adam_step");
}
