// In-launch BatchNorm folds: the producer of BN partial rows (part[nrows][2][C], fp64) also
// reduces them and applies the BN's stage-2 maths in its last-arriving blocks, so the separate
// fold launch (dk_bn_stats_from_partials_f32 / dk_bn_bwd_from_partials_f32, bn_fold_kernel)
// and its dependent-launch gap disappear from the step.
//
// Two levels, fixed order (deterministic run to run):
//   level 1: rows are grouped G at a time (G ~ sqrt(nrows)); the last block of a group to
//            finish (an agent-scope ticket per group and channel slice) folds the group's G
//            rows into grp[g][2][C].  Groups finish throughout the launch, so this work
//            hides under the blocks still running;
//   level 2: the last group folder of a slice (a second ticket) folds the ngroups group rows
//            and finalises the slice's channels (bn_finalize_channel: mean / std / invstd /
//            running statistics, or dgamma / dbeta / k12).
//
// Memory model (gfx950, cdna_hip_programming.md section 6, counter form): the partial rows and
// group rows are stored write-through (agent-scope relaxed atomic stores = global_store ... sc1)
// and every storing wave drains them (s_waitcnt vmcnt(0)) before the block's ticket; the ticket
// is an agent-scope atomic add; the last arriver executes an agent-scope acquire fence
// (buffer_inv sc1, dropping stale L1/L2 lines) and reads the rows with sc1 buffer loads.  No
// release fence (its L2 write-back in every block would cost more than the launch it saves).
// Tickets start at zero and the last arriver puts each back to zero, so the same words serve
// every launch on a stream.
#pragma once
#include "dk_common.h"

namespace dk {

struct FoldOut {
  int mode;  // 0: forward statistics, 1: backward coefficients, 2: plain sums
  double count;
  float eps, momentum;
  int first;
  float *mean, *std_, *invstd, *run_mean, *run_std;  // mode 0
  float *dgamma, *dbeta, *k12;                        // mode 1
  double* sums;                                       // mode 2: [2][C]
};

// Stage 2 of one channel from its totals (layers/batch_norm.py:76-89 forward, :147-171 backward).
__device__ __forceinline__ void bn_finalize_channel(int c, int C, double s, double q, const FoldOut& o) {
  if (o.mode == 0) {
    const double mean = s / o.count;
    double var = q / o.count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float meanf = (float)mean;
    const float stdf = sqrtf((float)var + o.eps);
    o.mean[c] = meanf;
    o.std_[c] = stdf;
    o.invstd[c] = 1.0f / stdf;
    if (o.run_mean) {
      if (o.first) {
        o.run_mean[c] = meanf;
        o.run_std[c] = stdf;
      } else {
        o.run_mean[c] = o.momentum * o.run_mean[c] + (1.0f - o.momentum) * meanf;
        o.run_std[c] = o.momentum * o.run_std[c] + (1.0f - o.momentum) * stdf;
      }
    }
  } else if (o.mode == 1) {
    o.dgamma[c] = (float)q;
    o.dbeta[c] = (float)s;
    o.k12[c] = (float)(s / o.count);
    o.k12[C + c] = (float)(q / o.count);
  } else {
    o.sums[c] = s;
    o.sums[C + c] = q;
  }
}

// Write-through (sc1) stores / loads for rows handed between blocks of one launch.
__device__ __forceinline__ void pub_store(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double pub_load(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct FoldTail {
  FoldOut o;
  const double* part;  // [nrows][2][C]: the rows this launch writes (nullptr: no in-launch fold)
  double* grp;         // [ngroups][2][C] scratch
  unsigned* tickets;   // [ngroups * nslices + nslices] zeroed words (left zero)
  int nrows, C, G, ngroups, nslices;
};

constexpr int kFoldBatch = 16;  // sc1 loads in flight per thread (one round trip for <= 16 rows per lane)

// Sum rows [r0, r0 + n) of src[.][2][C] over channels [c0, c0 + nc) (c0, nc, C even) and call
// out(c, S, Q) for each channel (threads t < chunk width).  All NT threads call it.  Thread
// (pair p, lane l) owns the 16-byte pair p of a channel chunk (S pairs, then Q pairs) and sums
// rows l, l + L, ... in order; the L lane sums are then added in lane order.
template <int NT, class Out>
__device__ void fold_block(double2* red, const double* src, int r0, int n, int C, int c0, int nc, Out out) {
  double* const tot = reinterpret_cast<double*>(red);  // [2][chunk] totals, after the lane sums
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(src + (size_t)r0 * 2 * C, (uint32_t)((size_t)n * 2 * C * 8));
  for (int ch0 = 0; ch0 < nc; ch0 += NT) {
    const int cw = min(NT, nc - ch0);  // channels (= 16-byte pairs) in this chunk
    const int half = cw >> 1;
    const int L = NT / cw;
    const int p = tid % cw, l = tid / cw;
    const int run = p / half;
    const int cc = c0 + ch0 + 2 * (p - run * half);
    double2 acc = {0.0, 0.0};
    if (l < L) {
      const uint32_t base = (uint32_t)((run * C + cc) * 8), stride = (uint32_t)(2 * C * 8);
      for (int r = l; r < n; r += L * kFoldBatch) {
        double2 v[kFoldBatch];
#pragma unroll
        for (int k = 0; k < kFoldBatch; ++k) {
          const int rr = r + k * L;
          const uint32_t off = rr < n ? base + (uint32_t)rr * stride : kOOBBytes;
          v[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
        }
#pragma unroll
        for (int k = 0; k < kFoldBatch; ++k) {
          acc.x += v[k].x;
          acc.y += v[k].y;
        }
      }
    }
    red[tid] = acc;
    __syncthreads();
    double2 s = acc;
    if (tid < cw) {
      for (int k = 1; k < L; ++k) {
        s.x += red[k * cw + tid].x;
        s.y += red[k * cw + tid].y;
      }
    }
    __syncthreads();
    if (tid < cw) {
      const int j = 2 * (tid - run * half);
      tot[run * cw + j] = s.x;
      tot[run * cw + j + 1] = s.y;
    }
    __syncthreads();
    if (tid < cw) out(c0 + ch0 + tid, tot[tid], tot[cw + tid]);
    __syncthreads();
  }
}

// Called by every thread of a block after it has stored (pub_store) its partial row `row` for
// channels [c0, c0 + nc) of slice `slice`.  Returns in every block; the last ones fold.
// red: >= NT double2 of LDS the block no longer needs (the wrapper below declares its own).
template <int NT>
__device__ void fold_tail(const FoldTail& f, int row, int c0, int nc, int slice, double2* red) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are done
  __syncthreads();
  const int g = row / f.G;
  const int r0 = g * f.G, n = min(f.G, f.nrows - r0);
  if (threadIdx.x == 0) {
    unsigned* t = f.tickets + g * f.nslices + slice;
    const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1u == (unsigned)n;
    if (last) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const FoldOut& o = f.o;
  const int C = f.C;
  if (f.ngroups == 1) {
    fold_block<NT>(red, f.part, r0, n, C, c0, nc, [&](int c, double s, double q) { bn_finalize_channel(c, C, s, q, o); });
    return;
  }
  double* gr = f.grp + (size_t)g * 2 * C;
  fold_block<NT>(red, f.part, r0, n, C, c0, nc, [&](int c, double s, double q) {
    pub_store(gr + c, s);
    pub_store(gr + C + c, q);
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* t = f.tickets + f.ngroups * f.nslices + slice;
    const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1u == (unsigned)f.ngroups;
    if (last) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  fold_block<NT>(red, f.grp, 0, f.ngroups, C, c0, nc, [&](int c, double s, double q) { bn_finalize_channel(c, C, s, q, o); });
}

template <int NT>
__device__ void fold_tail(const FoldTail& f, int row, int c0, int nc, int slice) {
  __shared__ double2 red[NT];  // fold_block's lane sums / channel totals (16 * NT bytes)
  fold_tail<NT>(f, row, c0, nc, slice, red);
}

// Host side: an armed partials buffer (dk_bn_fold_arm_*).  fold_take() hands the arming to the
// launch that writes `part` (nrows rows of C channels in nslices channel slices), filling `ft`;
// false (ft.part = nullptr) when nothing is armed for it or the scratch is too small.
bool fold_take(const void* part, int nrows, int C, int nslices, FoldTail* ft);
// The status an entry point returns after a launch that took an arming (DK_FOLDED on success).
int fold_status(int rc, const FoldTail& ft);

}  // namespace dk
