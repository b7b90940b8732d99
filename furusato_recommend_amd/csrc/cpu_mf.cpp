// Host (CPU) training step of configuration C1 — BASELINE configs[0]:
// "model/MF.py BPR, synthetic 5-core 10K x 1K / 50K-edge graph, d=32, CPU
// single-process".  One stageOne of model/MF.py:35-112 (bpr_loss :62-79,
// stageOne :88-94) with the reference's torch.optim.Adam (:42) over the
// whole table, on host arrays:
//
//   s_b   = <u_b, n_b> - <u_b, p_b>
//   loss  = mean_b softplus(s_b)               (torch softplus, threshold 20)
//   reg   = 0.5 (|U|^2 + |P|^2 + |N|^2) / B    (the gathered rows, duplicates counted)
//   total = loss + decay reg
//   G     = d total / d table                  (sigmoid(s_b) / B on the score
//                                              difference, decay / B on each
//                                              gathered row; repeated ids add)
//   Adam(lr, betas (0.9, 0.999), eps 1e-8) on every row (rows outside the
//   batch have G = 0 and still move with their moments, as torch's do).
//
// The gradient is accumulated in batch order on one thread (deterministic);
// the dense Adam and the gradient clear run on n_threads threads over row
// blocks.  The Adam arithmetic is the device kernels' (adam1, common.h).
// mirec_cpu_bpr_step = mirec_cpu_bpr_grad + mirec_cpu_adam; the two halves
// are exported for the host data-parallel step (dist.HostDataParallel: the
// gradient is all-reduced between them).
#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "mirec.h"

namespace {

inline void adam_host(float &p, float &m, float &v, float g, const mirec_adam_hparams_t &h) {
  m = std::fma(h.one_minus_beta1, g - m, m);
  v = std::fma(v, h.beta2, h.one_minus_beta2 * (g * g));
  const float denom = std::sqrt(v) / h.bc2_sqrt + h.eps;
  p = std::fma(h.neg_step_size, m / denom, p);
}

template <typename F>
void parallel_rows(int64_t n, int n_threads, F &&f) {
  const int nt = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::min(std::max(n_threads, 1), 64), (n + 65535) / 65536));
  std::vector<std::thread> th;
  for (int w = 1; w < nt; ++w) th.emplace_back([&, w] { f(n * w / nt, n * (w + 1) / nt); });
  f(0, n / nt);
  for (auto &x : th) x.join();
}

}  // namespace

extern "C" int mirec_cpu_bpr_grad(const float *table, float *grad, int64_t n_rows, int32_t dim,
                                  int64_t item_offset, const int32_t *users, const int32_t *pos,
                                  const int32_t *neg, int64_t batch, float decay,
                                  float grad_scale, float *loss_out, int32_t n_threads) {
  if (!table || !grad || n_rows <= 0 || dim <= 0 || item_offset < 0 || item_offset > n_rows ||
      batch <= 0 || !users || !pos || !neg)
    return MIREC_ERR_ARG;
  const int64_t d = dim;
  for (int64_t b = 0; b < batch; ++b) {
    if (users[b] < 0 || users[b] >= item_offset || pos[b] < 0 || neg[b] < 0 ||
        item_offset + pos[b] >= n_rows || item_offset + neg[b] >= n_rows)
      return MIREC_ERR_RANGE;
  }
  parallel_rows(n_rows * d, n_threads, [&](int64_t a, int64_t b) {
    std::fill(grad + a, grad + b, 0.f);
  });
  const float inv_b = 1.f / (float)batch * grad_scale;
  const float rc = decay * inv_b;
  double loss = 0.0, reg = 0.0;
  for (int64_t b = 0; b < batch; ++b) {
    const float *u = table + (int64_t)users[b] * d;
    const float *p = table + (item_offset + pos[b]) * d;
    const float *q = table + (item_offset + neg[b]) * d;
    float sp = 0.f, sn = 0.f, ru = 0.f, rp = 0.f, rn = 0.f;
    for (int64_t c = 0; c < d; ++c) {
      sp += u[c] * p[c];
      sn += u[c] * q[c];
      ru += u[c] * u[c];
      rp += p[c] * p[c];
      rn += q[c] * q[c];
    }
    const float s = sn - sp;
    loss += s > 20.f ? (double)s : std::log1p(std::exp((double)s));
    reg += (double)ru + rp + rn;
    const float cs = inv_b / (1.f + std::exp(-s));  // d loss / d s
    float *gu = grad + (int64_t)users[b] * d;
    float *gp = grad + (item_offset + pos[b]) * d;
    float *gn = grad + (item_offset + neg[b]) * d;
    for (int64_t c = 0; c < d; ++c) {
      const float uc = u[c], pc = p[c], qc = q[c];
      gu[c] += cs * (qc - pc) + rc * uc;
      gp[c] += rc * pc - cs * uc;
      gn[c] += cs * uc + rc * qc;
    }
  }
  if (loss_out)
    *loss_out = (float)(loss / (double)batch + (double)decay * 0.5 * reg / (double)batch);
  return MIREC_OK;
}

extern "C" int mirec_cpu_adam(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                              int64_t n, const mirec_adam_hparams_t *h, int32_t n_threads) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !h || n < 0) return MIREC_ERR_ARG;
  parallel_rows(n, n_threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) adam_host(param[i], exp_avg[i], exp_avg_sq[i], grad[i], *h);
  });
  return MIREC_OK;
}

extern "C" int mirec_cpu_bpr_step(float *table, float *exp_avg, float *exp_avg_sq, float *grad,
                                  int64_t n_rows, int32_t dim, int64_t item_offset,
                                  const int32_t *users, const int32_t *pos, const int32_t *neg,
                                  int64_t batch, float decay, const mirec_adam_hparams_t *h,
                                  float *loss_out, int32_t n_threads) {
  if (!exp_avg || !exp_avg_sq || !h) return MIREC_ERR_ARG;
  const int rc = mirec_cpu_bpr_grad(table, grad, n_rows, dim, item_offset, users, pos, neg, batch,
                                    decay, 1.f, loss_out, n_threads);
  if (rc != MIREC_OK) return rc;
  return mirec_cpu_adam(table, grad, exp_avg, exp_avg_sq, n_rows * (int64_t)dim, h, n_threads);
}
