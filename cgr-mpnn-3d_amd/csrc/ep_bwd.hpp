// Fused layer-backward epilogue of the dm GEMM (gemm_b3nt_kernel, kTile epilogues): one launch
// per layer computes dm = dpre_l W_l AND the layer below's dpre (the reverse of GNN.py:134-141):
//
//   da[v]       = sum_{src(e) = v} dm[e]
//   dh_l[i]     = da[dst(i)] - dm[rev(i)]
//   dpre_{l-1}  = dh_l * keep/(1-p) * act'(pre)        (or the edge init's dpre0, bwd_rows.hpp)
//
// The GEMM's A rows are gathered through rev (LdGatherRows), so its output row r is dm[rev(r)].
// With reverse-paired edges (graph prep's status bit 2 clear: src(e ^ 1) == dst(e), the CGR edge
// order of graph_features.py:184-195) {rev(i) : dst(i) = v} == {e : src(e) = v}: the dm rows
// summed into da[v] are exactly the output rows of v's dst segment, which is contiguous in the
// dst-sorted row order.  So the tile sums each dst segment from its accumulators in LDS, turns
// every row r into dh = da - C[r] in place and applies the activation backward -- da and dm
// never reach memory.  Segments crossing a tile boundary (at most one at each end) add their
// partial sums atomically to `dag` (two contributors: order-independent, so deterministic for
// in-degrees <= rows per tile + 1) and store their raw rows to a.dm; bwd_seg_fixup (kernels.hip)
// completes those rows after the GEMM.  Unpaired edge lists store every row raw and the fixup does
// the whole src-CSR form.
#pragma once

#include "bwd_rows.hpp"
#include "common.hpp"

namespace cgr {

template <bool EDGE_INIT>
struct EpLayerBwdSeg {
  static constexpr bool kSeg = false;
  static constexpr bool kTile = true;
  LayerBwdArgs a;     // the layer below (a.dpre written)
  float* raw;         // [M, Hp] = a.dm: the raw rows of crossing segments, for the fixup
  const int* dst_s;   // [M] node of each (dst-sorted) row
  float* dag;         // [nodes, Hp] crossing-segment partial sums of da (zero on entry)
  const int* status;  // graph prep's status word
  int M, N;           // rows (edges), columns (hidden)

  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  typedef RowOps Pre;
  // operands of row r, columns c..c+3 (unconditional loads from clamped in-bounds addresses)
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const int rr = r < M ? r : M - 1;
    const int cc = c < N ? c : ((N - 1) & ~3);
    return bwd_row_loads<EDGE_INIT>(a, rr, cc);
  }

  // C: the tile's accumulators [BM][LDC] in LDS (column j of the tile = output column n0 + j);
  // sd[q]: dst of rows m0 - 1 + q (q < BM + 2; distinct negative sentinels outside [0, M)),
  // followed by 16 floats of scratch;
  // pv: pre4 of the items (r, c4) = (q / C4, q % C4), q = tid + it * NT
  template <int BM, int BN, int NT, int LDC, int EIT>
  __device__ __forceinline__ void tile(const Pre (&pv)[EIT], float* C, const int* sd, int m0,
                                       int n0, int tile_id, int tid) const {
    constexpr int C4 = BN / 4, NCH = BM / 16;
    const int nrow = min(BM, M - m0);
    const bool paired = (*status & 4) == 0;
    if (paired) {
      // thread (16-row chunk, float4 column): every segment that STARTS in its chunk (running
      // past the chunk's end as needed) and, for chunk 0, the head segment begun in the
      // previous tile -- the forward's EpLayerSeg walk
      for (int q = tid; q < NCH * C4; q += NT) {
        const int ch = q / C4, c4 = q - ch * C4;
        const int col = n0 + 4 * c4;
        if (col >= N) continue;
        int s = 16 * ch;
        const int end = min(16 * ch + 16, nrow);
        if (ch > 0)
          while (s < end && sd[s + 1] == sd[s]) ++s;
        while (s < end) {
          const int v = sd[s + 1];
          float4 da = f4zero();
          int r = s;
          for (; r < nrow && sd[r + 1] == v; ++r)
            da = f4add(da, *reinterpret_cast<const float4*>(&C[r * LDC + 4 * c4]));
          const bool head = s == 0 && sd[0] == v, tail = r == nrow && sd[nrow + 1] == v;
          if (head || tail) {
            float* g = dag + (int64_t)v * a.Hp + col;
            atomicAdd(g, da.x);
            atomicAdd(g + 1, da.y);
            atomicAdd(g + 2, da.z);
            atomicAdd(g + 3, da.w);
          } else {
            for (int k = s; k < r; ++k) {
              float4* cp = reinterpret_cast<float4*>(&C[k * LDC + 4 * c4]);
              *cp = f4sub(da, *cp);
            }
          }
          s = r;
        }
      }
      __syncthreads();
    }
    // rows of crossing segments (or every row, unpaired): raw dm[rev(r)] for the fixup; all
    // others: dh -> the activation backward
    const int vh = sd[0] == sd[1] ? sd[0] : -3;             // head segment's node, if any
    const int vt = sd[nrow] == sd[nrow + 1] ? sd[nrow] : -3;  // tail segment's node, if any
    const uint64_t key = (!EDGE_INIT && a.thresh) ? *a.seed : 0;
    float dsig = 0.f;
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      const int q = tid + it * NT;
      if (q < BM * C4) {
        const int r = q / C4, c4 = q - r * C4;
        const int col = n0 + 4 * c4;
        if (r < nrow && col < N) {
          const float4 x = *reinterpret_cast<const float4*>(&C[r * LDC + 4 * c4]);
          const int v = sd[r + 1];
          const int64_t i = m0 + r;
          if (!paired || v == vh || v == vt)
            *reinterpret_cast<float4*>(raw + i * a.Hp + col) = x;
          else
            bwd_row_apply<EDGE_INIT>(a, i, col, x, key, dsig, pv[it]);
        }
      }
    }
    if (!EDGE_INIT && a.dsig_part) {  // this workgroup's slot of the learnable-skip partials
      static_assert(NT / 64 <= 16, "reduction scratch: 16 floats after sd (B3NtShape)");
      float* red = reinterpret_cast<float*>(const_cast<int*>(sd) + BM + 2);
      dsig = wave_sum(dsig);
      if ((tid & 63) == 0) red[tid >> 6] = dsig;
      __syncthreads();
      if (tid == 0) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w];
        a.dsig_part[tile_id] = s;
      }
    }
  }
};

}  // namespace cgr
