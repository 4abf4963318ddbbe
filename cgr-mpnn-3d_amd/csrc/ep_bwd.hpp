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
// never reach memory.
//
// Segments crossing a row-tile boundary (at most one at each end of a tile) are completed inside
// the launch by the LAST of their contributing workgroups (cdna_hip_programming.md §6
// Guideline 16, counter form): each contributor hands over its partial sum -- a segment over two
// row tiles adds it atomically to `dag` (two addends onto zero: order-independent), one over
// three or more (a hub node: in-degree > rows per tile + 1) stores it write-through into a slot
// fixed by the data (`part`, slot_of below), which the completer sums in row-tile order, so every
// reduction is deterministic whatever the in-degree -- and
// stores the segment's raw rows write-through (sc1), publishes them (vmcnt drain, barrier: no
// release fence -- an agent-scope release writes back the XCD's L2, here full of the dpre rows
// just stored: the fenced form ran each GEMM 15-20 us longer) and draws a ticket from the
// segment's counter; the workgroup that draws the last ticket reads the partial sums and raw rows
// with sc1 loads (no acquire) and applies the activation backward to all of the segment's rows,
// then resets the counter and zeroes the segment's entries of the next layer's `dag` buffer (two
// buffers alternate by layer).  No workgroup waits for another.
//
// Unpaired edge lists (status bit 2) have no such locality: every workgroup stores its rows raw
// and draws a ticket from this launch's own grid counter (one per fused launch, all zeroed by the
// top layer's activation kernel; nothing resets them mid-backward, so one launch's counts can
// never leak into the next); the last K arrivers (K = unpaired_completers(grid) <= 16) wait
// until every ticket is drawn and complete the src-CSR form over the nodes v = rank (mod K),
// every column.  The wait always ends: workgroups are dispatched round-robin over the 8 XCDs of
// 32 CUs, so K <= 16 spinning workgroups can never hold every CU of any XCD, and every other
// workgroup (of this launch or of a kernel beside it) runs to its end without waiting -- a CU of
// the XCD an undispatched workgroup belongs to always frees up.  Should a wait still exceed the
// spin limit, the completer reports it (status bit 16, and the host-visible error word the
// Python side raises from: cgr_device_errors) and writes NaN instead of a partial da, so the
// gradients it feeds are visibly poisoned, never silently wrong.  (Round 3 ran the completion in
// the grid's last workgroup alone: 6.0 ms per launch at cfg2 against 52 us paired.)
#pragma once

#include <type_traits>

#include "bwd_rows.hpp"
#include "common.hpp"
#include "handoff.hpp"
#include "stamps.hpp"

namespace cgr {

// completers of the unpaired form: half the grid, at most 16 -- half of one XCD's 32 CUs, so the
// spinning completers can never occupy every CU an undispatched workgroup could be placed on
__host__ __device__ inline int unpaired_completers(int grid) {
  const int k = grid / 2;
  return k < 1 ? 1 : (k > 16 ? 16 : k);
}


template <bool EDGE_INIT>
struct EpLayerBwdSeg {
  static constexpr bool kSeg = false;
  static constexpr bool kTile = true;
  LayerBwdArgs a;      // the layer below (a.dpre written)
  float* raw;          // [M, Hp]: the raw rows of crossing segments (every row, unpaired)
  const int* dst_s;    // [M] node of each (dst-sorted) row
  const int* dst_ptr;  // [nodes + 1] dst CSR of the sorted rows
  const int* src_list;  // unpaired form: src CSR (src_ptr) of the sorted rows
  const int* src_ptr;
  float* dag;          // [nodes, Hp] crossing-segment partial sums of da (zero on entry)
  float* dag_next;     // the next layer's (or null): completed segments' entries zeroed
  float* part;         // [tiles, 2, BN] partials of segments over >= 3 row tiles (slot_of)
  int* cnt;            // [nodes * tiles_n] segment tickets (zero on entry, left zero)
  const int* status;   // graph prep's status word
  int M, N, nodes, tiles_n;
  int* gcnt;           // unpaired form: this launch's grid ticket counter (zero on entry)
  int* dev_err;        // host-visible error words (kDevErr*), or null
  int spin_limit;      // unpaired completers' wait bound (< 0: report at once; debug knob)
  // mean aggregation: a = segsum_dst(h) / deg, so dh gets da[dst] / deg(dst) (nullable: add)
  const float* dscale;

  struct Ctx {};
  __device__ __forceinline__ Ctx ctx(int) const { return Ctx{}; }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  typedef RowOps Pre;
  // operands of row r, columns c..c+3 (unconditional loads from clamped in-bounds addresses)
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const int rr = r < M ? r : M - 1;
    const int cc = c < N ? c : ((N - 1) & ~3);
    return bwd_row_loads<EDGE_INIT>(a, rr, cc);
  }

  // C: the tile's accumulators [BM][LDC] in LDS (column j of the tile = output column n0 + j);
  // sd[q]: dst of rows m0 - 1 + q (q < BM + 2; distinct negative sentinels outside [0, M)),
  // followed by 16 words of scratch; RPP > 0: thread tid < RPP * C4 owns the float4 column group
  // tid % C4 of rows tid / C4 + RPP * it; RPP == 0 (flat): pass it takes piece q = tid + NT * it
  // of the tile's BM x C4, row q / C4, column group q % C4; pv[it] holds pre4 of pass it's piece;
  // tile_id: this workgroup's tile (tm * tiles_n + tn)
  template <int BM, int BN, int NT, int LDC, int EIT, int RPP>
  __device__ __forceinline__ void tile(const Pre (&pv)[EIT], float* C, const int* sd, int m0,
                                       int n0, int tile_id, int tid) const {
    constexpr int C4 = BN / 4;
    constexpr bool FLAT = RPP == 0;
    const bool eact = FLAT || tid < RPP * C4;
    const int ec4 = FLAT ? 0 : (eact ? tid % C4 : 0), er0 = FLAT ? 0 : tid / C4;
    const int nrow = min(BM, M - m0);
    const bool paired = (*status & 4) == 0;
    int* scratch = const_cast<int*>(sd) + BM + 2;  // 16 words
    const int vh = sd[0] == sd[1] ? sd[0] : -3;               // head segment's node, if any
    const int vt = sd[nrow] == sd[nrow + 1] ? sd[nrow] : -3;  // tail segment's node, if any
    const uint64_t key = (!EDGE_INIT && a.thresh) ? *a.seed : 0;
    float dsig = 0.f;
    // one pass, every row independent: row r's dst segment [s, e) inside the tile from the
    // tile's segment-start mask (rows are dst-sorted; with paired edges its rows are exactly the
    // dm rows its node sums), da = the segment's sum in row order (the same for every row of the
    // segment), dh = da - dm[rev(r)] -> the activation backward.  A segment crossing a row tile
    // (or every row, unpaired) stores its raw rows for the completer, and its first row in the
    // tile hands over the partial sum.  One loop per activation (the switch outside the loop).
    const uint32_t* smask = reinterpret_cast<const uint32_t*>(sd + BM + 2 + 8);
    const uint64_t mlo = smask[0] | ((uint64_t)smask[1] << 32);
    const uint64_t mhi = smask[2] | ((uint64_t)smask[3] << 32);
    CGR_STAMP(4);
    auto rows = [&](auto Ac) {
      constexpr int A = decltype(Ac)::value;
#pragma unroll
      for (int it = 0; it < EIT; ++it) {
        int r, c4;
        if constexpr (FLAT) {
          const int q = tid + NT * it;
          if (q >= BM * C4) break;
          r = q / C4;
          c4 = q - r * C4;
        } else {
          r = er0 + RPP * it;
          c4 = ec4;
        }
        const int col = n0 + 4 * c4;
        if (!eact || r >= nrow || col >= N) continue;
        const float4 x = *reinterpret_cast<const float4*>(&C[r * LDC + 4 * c4]);
        const int64_t i = m0 + r;
        if (!paired) {
          sc1_store4(raw + i * a.Hp + col, x);
          continue;
        }
        const int v = sd[r + 1];
        const int s = seg_first(mlo, mhi, r), e = seg_end(mlo, mhi, r);
        const bool head = s == 0 && sd[0] == v, tail = e == nrow && sd[nrow + 1] == v;
        float4 da = f4zero();
        for (int k = s; k < e; ++k)
          da = f4add(da, *reinterpret_cast<const float4*>(&C[k * LDC + 4 * c4]));
        if (head || tail) {
          sc1_store4(raw + i * a.Hp + col, x);
          if (r == s) {
            const int b = dst_ptr[v], ee = dst_ptr[v + 1];
            if (seg_tiles(b, ee, BM) <= 2) {
              float* g = dag + (int64_t)v * a.Hp + col;
              atomicAdd(g, da.x);
              atomicAdd(g + 1, da.y);
              atomicAdd(g + 2, da.z);
              atomicAdd(g + 3, da.w);
            } else {
              const int slot = slot_of(m0 / BM, b / BM);
              sc1_store4(part + ((int64_t)tile_id * 2 + slot) * BN + 4 * c4, da);
            }
          }
        } else {
          if (dscale) da = f4scale(da, dscale[v]);
          bwd_row_apply<EDGE_INIT, A>(a, i, col, f4sub(da, x), key, dsig, pv[it]);
        }
      }
    };
    if (a.act == ACT_RELU) rows(std::integral_constant<int, ACT_RELU>{});
    else if (a.act == ACT_SILU) rows(std::integral_constant<int, ACT_SILU>{});
    else rows(std::integral_constant<int, -1>{});  // GELU and the rest (common.hpp)

    CGR_STAMP(5);
    // ---- hand-off: the last contributor of a crossing segment (or of the grid) completes it ----
    const int tn = tile_id % tiles_n;
    float dsig_c[2] = {0.f, 0.f};  // learnable-skip partials of the segments completed here
    int scratch_f0 = -1, scratch_f1 = -1;
    if (!paired || vh >= 0 || vt >= 0) {  // uniform over the workgroup
      // unpaired: slot grid + r belongs to completer rank r < K (written once, by it: two
      // workgroups' plain stores to one slot could land from two XCDs' L2s in either order); the
      // slots past the completers' are zeroed by their tiles
      if (!EDGE_INIT && !paired && a.dsig_part && tid == 0 &&
          tile_id >= unpaired_completers((int)gridDim.x))
        a.dsig_part[gridDim.x + tile_id] = 0.f;
      ep_vm_drain();  // this wave's partial-sum atomics and raw-row stores
      __syncthreads();
      if (tid == 0) {
        bool any = false;
        if (paired) {
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int v = k == 0 ? vh : (vt != vh ? vt : -3);
            int done = 0;
            if (v >= 0) {
              const int contributors =
                  (dst_ptr[v + 1] - 1) / BM - dst_ptr[v] / BM + 1;  // row tiles it touches
              const int t = __hip_atomic_fetch_add(&cnt[(int64_t)v * tiles_n + tn], 1,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              done = t == contributors - 1;
            }
            scratch[14 + k] = done ? v : -1;
            any = any || done;
          }
        } else {
          const int G = (int)gridDim.x, K = unpaired_completers(G);
          const int t = __hip_atomic_fetch_add(gcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          any = t >= G - K;
          scratch[14] = any ? t - (G - K) : -1;  // completer rank
          scratch[15] = -1;
        }
        (void)any;
      }
      __syncthreads();
      const int f0 = scratch[14], f1 = scratch[15];
      scratch_f0 = f0;
      scratch_f1 = f1;
      if (paired) {
        // every row of each completed segment x this tile's columns
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int v = k == 0 ? f0 : f1;
          if (v < 0) continue;
          const int ib = dst_ptr[v], ie = dst_ptr[v + 1];
          const int64_t gv = (int64_t)v * a.Hp;
          float ds = 0.f;
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // loads stay below the ticket
          // da of the segment per column into LDS (the tile's accumulators are dead): the atomic
          // sum of two partials, or the slots of every row tile in row order
          const int t0 = ib / BM, t1 = (ie - 1) / BM;
          float4* das = reinterpret_cast<float4*>(C);
          __syncthreads();  // previous segment's das reads done
          for (int c4 = tid; c4 < C4; c4 += NT) {
            float4 da = f4zero();
            if (t1 - t0 + 1 <= 2) {
              da = sc1_load4(dag + gv + n0 + 4 * c4);
            } else {
              for (int t = t0; t <= t1; ++t)
                da = f4add(da, sc1_load4(part + ((int64_t)(t * tiles_n + tn) * 2 + slot_of(t, t0)) *
                                                    BN + 4 * c4));
            }
            das[c4] = dscale ? f4scale(da, dscale[v]) : da;
          }
          __syncthreads();
          for (int q = tid; q < (ie - ib) * C4; q += NT) {
            const int i = ib + q / C4, col = n0 + 4 * (q % C4);
            if (col >= N) continue;
            const float4 da = das[q % C4];
            const float4 x = sc1_load4(raw + (int64_t)i * a.Hp + col);
            bwd_row_apply<EDGE_INIT>(a, i, col, f4sub(da, x), key, ds,
                                     bwd_row_loads<EDGE_INIT>(a, i, col));
          }
          dsig_c[k] = ds;
          if (dag_next)
            for (int c4 = tid; c4 < C4; c4 += NT)
              if (n0 + 4 * c4 < N)
                *reinterpret_cast<float4*>(dag_next + gv + n0 + 4 * c4) = f4zero();
          if (tid == 0) cnt[(int64_t)v * tiles_n + tn] = 0;
        }
      } else if (f0 >= 0) {
        // unpaired completer of rank f0: once every workgroup has drawn its ticket (its raw rows
        // are published), da[v] = sum_{src(e) = v} dm[e] = raw[rev(e)] and every row of v's dst
        // segment, for the nodes v = f0 (mod K), all columns
        const int G = (int)gridDim.x, K = unpaired_completers(G);
        if (tid == 0) {
          int spins = 0;
          bool late = spin_limit < 0;
          while (!late && __hip_atomic_load(gcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G) {
            if (++spins >= spin_limit) late = true;
            else __builtin_amdgcn_s_sleep(2);
          }
          if (late) {
            atomicOr(const_cast<int*>(status), 16);
            if (dev_err)
              __hip_atomic_store(dev_err + kDevErrUnpairedTimeout, 1, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
          }
          if (dev_err && f0 == 0)
            __hip_atomic_store(dev_err + kDevErrUnpairedSeen, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          scratch[13] = late ? 1 : 0;
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // loads stay below the wait
        // a completer that gave up waiting poisons what it writes (NaN), never a partial sum
        const float poison = scratch[13] ? __builtin_nanf("") : 0.f;
        const int C4all = a.Hp >> 2;
        const int64_t mine = nodes > f0 ? (nodes - f0 + K - 1) / K : 0;
        float ds = 0.f;
        for (int64_t q = tid; q < mine * C4all; q += NT) {
          const int v = f0 + K * (int)(q / C4all), col = 4 * (int)(q % C4all);
          float4 da = make_float4(poison, poison, poison, poison);
          for (int j = src_ptr[v], e = src_ptr[v + 1]; j < e; ++j)
            da = f4add(da, sc1_load4(raw + (int64_t)a.rev_s[src_list[j]] * a.Hp + col));
          if (dscale) da = f4scale(da, dscale[v]);
          for (int i = dst_ptr[v], e = dst_ptr[v + 1]; i < e; ++i) {
            const float4 x = sc1_load4(raw + (int64_t)i * a.Hp + col);
            bwd_row_apply<EDGE_INIT>(a, i, col, f4sub(da, x), key, ds,
                                     bwd_row_loads<EDGE_INIT>(a, i, col));
          }
        }
        dsig_c[0] = ds;
      }
    }

    CGR_STAMP(6);
    // learnable-skip partials, at positions fixed by the data (not by which workgroup finished
    // last, so their fixed-order sum is deterministic): slot tile_id = this tile's rows; slot
    // gridDim.x + t = the rows of the crossing segment that STARTS in tile t (written by its
    // completer; zero when none starts there).  Unpaired: everything is the completer's, in its
    // own tile slot (all other slots are zero, so the sum is exact whatever the completer).
    if (!EDGE_INIT && a.dsig_part) {
      static_assert(NT / 64 <= 8, "reduction scratch: words 0..7 after sd (B3NtShape)");
      float* red = reinterpret_cast<float*>(scratch);
      auto block_sum = [&](float x) {
        x = wave_sum(x);
        __syncthreads();  // scratch free (flags read, previous sum consumed)
        if ((tid & 63) == 0) red[tid >> 6] = x;
        __syncthreads();
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w];
        return s;
      };
      const float st = block_sum(dsig);
      if (tid == 0) a.dsig_part[tile_id] = st;
      const int f[2] = {scratch_f0, scratch_f1};
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (paired && f[k] >= 0) {
          const float sc = block_sum(dsig_c[k]);
          if (tid == 0)
            a.dsig_part[gridDim.x + (dst_ptr[f[k]] / BM) * tiles_n + tn] = sc;
        }
      if (paired) {
        const bool starts = vt >= 0 && dst_ptr[vt] >= m0;
        if (!starts && tid == 0) a.dsig_part[gridDim.x + tile_id] = 0.f;
      } else if (f[0] >= 0) {  // unpaired completer: its nodes' partial in the slot of its rank
        const float sc = block_sum(dsig_c[0]);
        if (tid == 0) a.dsig_part[gridDim.x + f[0]] = sc;
      }
    }
  }
};

}  // namespace cgr
