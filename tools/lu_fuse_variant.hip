// Stage II: batched dense LU with partial pivoting and the two triangular solves
// (reference: models/lu.py:26-35, torch.lu / torch.lu_solve on K[B,N,N]).
//
// Right-looking blocked LU (the ?getrf structure) in 128-column outer blocks, each split into two
// 64-column halves factored as 16-column panels (N <= 2048) or 8-column panels (N > 2048):
//   lu_panel_kernel        one workgroup per instance: the (N-k) x 16 (x 8) panel is factored in registers
//                          (pivot = first max |a| like LAPACK i?amax; the multipliers use a
//                          reciprocal like ?getf2), the row interchanges are applied to the
//                          half's other columns (?laswp), and U = L11^-1 A is solved for the
//                          panel rows inside the current half; lu_panel_global_kernel is the
//                          same column steps with the panel in HBM / L2 (more than 10240 rows).
//   lu_update_block_kernel A -= L21 U12 on the columns of the current half right of the panel
//                          (lu_update_block_vec_kernel<NB, W> when the width is 48, 32 or 16).
// per 128-column block: first half factored; its interchanges + U12 on the second half
// (lu_swap_kernel<64, true>); the second half's rank-64 update (lu_trail_kernel, cmax); second
// half factored; its interchanges on the first half; the block's 128 interchanges composed into
// one row permutation (lu_block_perm_kernel), applied right of the block by the trailing update's
// gathered loads and left of it at the end, all blocks in one pass (lu_left_compose_kernel +
// lu_left_apply_kernel; N > 2048: per block, lu_swap_kernel<128, false>); L11^-1 (lu_linv_kernel); then
//   lu_trail128_kernel     U12 = L11^-1 A12 (MFMA prologue) and A22 -= L21 U12 at rank 128 on fp32
//                          MFMA (v_mfma_f32_32x32x2f32): 128-column strips streamed in 32-row
//                          steps, A22 read + written once per 128 columns.  With the left
//                          interchanges deferred, strip 0 (the next block's columns) runs on the
//                          caller's stream and the other strips on a side stream, beside the
//                          next block's factorization (look-ahead, lu_factor_blocks).
// lu_solve_kernel: one workgroup per instance; P b, then blocked forward (unit L) and backward
// (U) substitution: 64-row blocks, prefix dot products over coalesced row segments, the 64x64
// diagonal block solved inside one wave.
//
// Rounding (r04): every multiply-subtract of the VALU paths (panel rank-1 updates, in-half updates,
// the in-panel and TRSM substitutions, the solve's diagonal blocks) is one fmaf, a single rounding
// per term as in LAPACK's ?getf2 / ?trsm / ?gemm on FMA hardware (the library builds with
// -ffp-contract=off so that the elementwise kernels keep the reference's mul-then-add rounding; the
// LU has no such reference order, and the r03 two-rounding form measured a 1.3-1.8x larger
// factorisation backward error than MKL's sgetrf on the KKT matrices: tools/lu_diag.py).
//
// Pivots are stored 1-based, LAPACK / torch.linalg.lu_factor convention (row i was swapped with
// row piv[i]-1), so (LU, piv) also feeds torch.linalg.lu_solve.  info[b] = first i+1 with a zero
// pivot (0 = non-singular), LAPACK convention.
#include <algorithm>
#include <cstdlib>
#include <new>
#include <type_traits>

#include "common.h"

namespace iadmm {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
IADMM_DEV void vm_wait() {  // s_waitcnt vmcnt(N), other counters untouched (gfx9 encoding)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Wave-wide argmax of (best, bi): the largest value, the smallest index among equal values (the
// pivot rule of LAPACK i?amax).  The rule is a total order, so the result does not depend on the
// pairing order: DPP within 16-lane rows (quad_perm xor 1, xor 2, row_half_mirror, row_mirror) and
// gfx950's v_permlane16/32_swap across rows -- VALU-latency steps instead of six ds_bpermute LDS
// round trips per column (r04).
IADMM_DEV void wave_argmax(float& best, int& bi) {
  auto comb = [&](int ov, int oi) {
    const float v = __int_as_float(ov);
    if (v > best || (v == best && oi < bi)) { best = v; bi = oi; }
  };
  auto dpp = [&](int ctrl) {
    const int bv = __float_as_int(best);
    int ov, oi;
    switch (ctrl) {  // (the DPP control must be an immediate)
      case 0: ov = __builtin_amdgcn_mov_dpp(bv, 0xB1, 0xF, 0xF, false); oi = __builtin_amdgcn_mov_dpp(bi, 0xB1, 0xF, 0xF, false); break;
      case 1: ov = __builtin_amdgcn_mov_dpp(bv, 0x4E, 0xF, 0xF, false); oi = __builtin_amdgcn_mov_dpp(bi, 0x4E, 0xF, 0xF, false); break;
      case 2: ov = __builtin_amdgcn_mov_dpp(bv, 0x141, 0xF, 0xF, false); oi = __builtin_amdgcn_mov_dpp(bi, 0x141, 0xF, 0xF, false); break;
      default: ov = __builtin_amdgcn_mov_dpp(bv, 0x140, 0xF, 0xF, false); oi = __builtin_amdgcn_mov_dpp(bi, 0x140, 0xF, 0xF, false); break;
    }
    comb(ov, oi);
  };
  dpp(0);
  dpp(1);
  dpp(2);
  dpp(3);
  {
    const auto v = __builtin_amdgcn_permlane16_swap(__float_as_int(best), __float_as_int(best), false, false);
    const auto i = __builtin_amdgcn_permlane16_swap(bi, bi, false, false);
    comb(v[0], i[0]);
    comb(v[1], i[1]);
  }
  {
    const auto v = __builtin_amdgcn_permlane32_swap(__float_as_int(best), __float_as_int(best), false, false);
    const auto i = __builtin_amdgcn_permlane32_swap(bi, bi, false, false);
    comb(v[0], i[0]);
    comb(v[1], i[1]);
  }
}

constexpr int kNB = 16;
constexpr int kPanelMaxM = 8;      // panel rows per thread: N <= 8 * 256 (12 rows spilled 782 VGPRs)
constexpr int kBigNB = 8;          // panel width above N = 8 * 256
constexpr int kBigThreads = 1024;  // panel workgroup size above N = 8 * 256
constexpr int kBigMaxM = 10;       // rows per thread there: N <= 10 * 1024 (12 spills at 128 VGPRs)
constexpr int kLuMaxN = 36736;     // = lu_solve's LDS limit; panels past 10240 rows run from HBM
constexpr int kLuMaxHbmN = 46340;  // above kLuMaxN: x in HBM, interchanges as a pass (N * N < 2^31)
constexpr int kLuThreads = 256;
constexpr int kUpdRows = 64;
constexpr int kSolveBlk = 64;
constexpr int kSolveThreads = 256;  // (512 measured slower: 4.3 vs 3.5 ms per solve at B = 1024, N = 2000)
constexpr int kBlk = 64;          // outer block width = rank of the trailing update
constexpr int kTC = 128;          // trailing update: columns per workgroup strip
constexpr int kTRS = 64;          //   rows per pipeline step
constexpr int kTRW = 1024;        //   rows per workgroup
constexpr int kTS = kBlk + 4;     //   LDS row stride of the staged U12^T / -L21 blocks
constexpr int kTrailThreads = 512;
// LDS of lu_trail_kernel<.., TCW>: U12^T [TCW][kTS], -L21 [kTRS][kTS] (one buffer: it is rewritten
// only after the step's barrier), Cin / Cout [kTRS][TCW + 8].  TCW = 64 (the mid update): 70 KB, so
// under the look-ahead it fits on a CU beside one lu_trail128_kernel workgroup (r04; the r03 layout,
// 136 KB for any TCW, waited for whole CUs to drain).
template <int TCW>
constexpr size_t trail_lds() { return ((size_t)(TCW + kTRS) * kTS + 2 * (size_t)kTRS * (TCW + 8)) * sizeof(float); }
constexpr size_t kTrailLds = trail_lds<kTC>();

// The net row permutation of n interchanges (row base + j <-> pv[j], in order, ?laswp):
// afterwards row rowid[i] holds what row cur[i] held before, for i < *cnt (<= 2n <= 64 NS; rowid[i] =
// base + i for i < n).  Built by one wave with both lists in registers (entry i = lane i % 64 of slot
// i / 64): per interchange a ballot search over the live slots and lane-indexed reads and writes,
// no LDS round trip (r04: the LDS-resident lists cost ~500 cycles per interchange, ~30 us for a
// 128-row block); the lists go to LDS once at the end.  The caller moves each column with all loads
// before all stores, one memory latency instead of n.  NS = 4: a block (n <= 128); NS = 8: n <= 256.
// (wave: the wave that builds; sync = false: no closing barrier -- only that wave reads the lists)
template <int NS = 4>
IADMM_DEV void build_row_perm(const int* pv, int base, int n, int* rowid, int* cur, int* cnt, int wave = 0,
                              bool sync = true) {
  const int lane = threadIdx.x & 63;
  if ((int)(threadIdx.x >> 6) == wave) {
    int rw[NS], cr[NS], pvr[NS / 2];
#pragma unroll
    for (int s = 0; s < NS; ++s) rw[s] = cr[s] = base + 64 * s + lane;
#pragma unroll
    for (int s = 0; s < NS / 2; ++s) pvr[s] = pv[min(64 * s + lane, n - 1)];
    int c = n;
    for (int j = 0; j < n; ++j) {
      int pj = pvr[0];
#pragma unroll
      for (int s = 1; s < NS / 2; ++s) pj = s == (j >> 6) ? pvr[s] : pj;
      const int p = __builtin_amdgcn_readlane(pj, j & 63);
      if (p == base + j) continue;
      int found = -1;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (found < 0 && 64 * s < c) {
          const unsigned long long m = __ballot(rw[s] == p && 64 * s + lane < c);
          if (m) found = 64 * s + __ffsll((long long)m) - 1;
        }
      }
      if (found < 0) {
        found = c++;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s == (found >> 6) && lane == (found & 63)) { rw[s] = p; cr[s] = p; }
      }
      const int sj = j >> 6, sf = found >> 6;
      int vj = cr[0], vf = cr[0];  // cr[sj], cr[sf] for wave-uniform run-time slots (registers only)
#pragma unroll
      for (int s = 1; s < NS; ++s) {
        vj = s == sj ? cr[s] : vj;
        vf = s == sf ? cr[s] : vf;
      }
      const int tj = __builtin_amdgcn_readlane(vj, j & 63), tf = __builtin_amdgcn_readlane(vf, found & 63);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s == sj && lane == (j & 63)) cr[s] = tf;
        if (s == sf && lane == (found & 63)) cr[s] = tj;
      }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (64 * s + lane < c) { rowid[64 * s + lane] = rw[s]; cur[64 * s + lane] = cr[s]; }
    if (lane == 0) *cnt = c;
  }
  if (sync) __syncthreads();
}

// The (N-k0) x 16 panel lives in registers: thread t owns rows t + 256 m (m < M), 16 columns
// each.  Per column j: argmax |a| (thread scan, wave shuffle tree; first index on ties); each
// wave's winner writes its whole row to LDS beside the wave's |a| and index, the owner of row j
// writes row j; one barrier; every thread then combines the waves' winners itself, the owners of
// rows j and p take their new rows from LDS, and every thread scales its rows below j by the
// reciprocal and applies the rank-1 update in registers.  One barrier per column (r02/r03: three,
// with one thread combining the waves between two of them); the LDS is double-buffered by column
// parity.  M = ceil((N-k0)/256) rounded up to the next instantiated size.
template <int NB>
IADMM_DEV float col_of(const float (&row)[NB], int j) {  // row[j] for a run-time j, registers only
  float v = row[0];
#pragma unroll
  for (int c = 1; c < NB; ++c) v = c == j ? row[c] : v;
  return v;
}

// After a panel [k0, k0 + nb) is factored (L11 in LDS, its interchanges in pvs): the row
// interchanges (?laswp) on the columns of the current 64-column block outside the panel (the
// columns left and right of the block get the whole block's interchanges at once in
// lu_swap_kernel), then U = L11^-1 A on the panel rows for the columns [k0 + nb, cend) of the block
// (unit lower forward substitution, one column per thread with its loads issued before the
// substitution).
// Ut (FUSE panels, may be null): the U rows also go to Ut[i][c - k0 - nb] (LDS) for the slab update.
template <int NB>
IADMM_DEV void panel_finish(float* Ab, int N, int K0, int k0, int nb, int cend, float (*L11)[NB + 1], const int* pvs,
                            int* prow, int* pcur, int* pcnt, float (*Ut)[3 * NB] = nullptr) {
  const int tid = threadIdx.x;
  build_row_perm(pvs, k0, nb, prow, pcur, pcnt);  // (its barrier also publishes L11)
  {
    const int cnt = *pcnt;
    const int col = K0 + tid;
    if (col < cend && (col < k0 || col >= k0 + nb)) {
      float v[2 * NB];
#pragma unroll
      for (int i = 0; i < 2 * NB; ++i) v[i] = Ab[(size_t)pcur[min(i, cnt - 1)] * N + col];  // (unconditional loads)
#pragma unroll
      for (int i = 0; i < 2 * NB; ++i)
        if (i < cnt) Ab[(size_t)prow[i] * N + col] = v[i];
    }
  }
  __syncthreads();  // the substitution's column owners differ from the interchanges'
  const int c = k0 + nb + tid;
  if (c < cend) {
    float x[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) x[i] = Ab[(size_t)(k0 + min(i, nb - 1)) * N + c];
#pragma unroll
    for (int i = 1; i < NB; ++i) {
      float s = x[i];
#pragma unroll
      for (int l = 0; l < i; ++l) s = fmaf(-L11[i][l], x[l], s);
      x[i] = s;
      // (one row's L11 reads at a time: hoisting all 120 of them would cost the panel kernels
      // their fourth workgroup per CU)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (i < nb) Ab[(size_t)(k0 + i) * N + c] = x[i];
    if (Ut) {
#pragma unroll
      for (int i = 0; i < NB; ++i) Ut[i][tid] = x[i];
    }
  }
}

// Panel shapes: <M, 16, 256> (2 workgroups per CU) for N <= 8 * 256 = 2048; above that
// <M, 8, 1024>: one 16-wave workgroup per CU holds up to 10 * 1024 = 10240 panel rows in
// registers (an 8-wide panel keeps 10 rows per thread within the 128 VGPRs a 1024-thread
// workgroup allows; 12 rows spill), so the pivot search still sees the whole column without
// leaving registers.
// DIAG (tools/lupanelbench.hip only): 1 = no column steps (identity interchanges), 2 = no
// panel_finish, 3 = neither (the panel's load and store alone).
// FUSE (r06; 16-wide staged panels of a full 64-column half): the half's in-half updates happen
// inside its panels instead of in separate launches.  Right-looking, panel q's rank-16 update went to
// every row below it on the half's later columns; here it is split by rows:
//   * rows [k0 + 16, cend) -- the later panels' own rows, <= 48 -- right after panel q, by the
//     threads that hold those rows' L in registers, with U from panel_finish's LDS copy ("slab
//     update"), so that the later panels' U rows come out of panel_finish as before;
//   * rows >= cend: panel j applies the updates of all earlier panels q < j to its own 16 columns as
//     its rows arrive (L of the half's earlier columns streamed through the LDS stage, U rows from
//     HBM), q = 0 .. j - 1 in order.
// Every element gets the same fmaf sequence as from lu_update_block_vec_kernel (the factors are bit
// for bit those of the separate updates), and the half's columns move through HBM once per panel
// instead of once more per update: 304 -> 224 column passes per half.
template <int M, int NB, int NT, int DIAG = 0, bool FUSE = false, int JQ = 0>
__global__ __launch_bounds__(NT, NT <= 256 ? (M <= 6 ? 4 : 2) : 1) void lu_panel_kernel(int N, int K0, int k0, int cend, float* A,
                                                                         int* piv, int* info) {
  constexpr int kNB = NB, kLuThreads = NT, NWV = NT / 64;
  // per column, double-buffered (index j & 1) so a column costs one barrier: each wave's
  // candidate pivot row, its |a| and index, and row j before the exchange
  __shared__ float cand[2][NWV][kNB];
  __shared__ float rowj[2][kNB];
  __shared__ float L11[kNB][kNB + 1];
  __shared__ float rv[2][NWV];
  __shared__ int ri[2][NWV];
  __shared__ int pvs[kNB], prow[2 * kNB], pcur[2 * kNB], pcnt[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  const int R = N - k0;
  const int nb = min(kNB, R);
  const bool vec = nb == kNB && (N % 4) == 0 && aligned16(Ab);

  float a[M][kNB];
  // STAGED (16-wide panels on 256 threads, 16-B aligned rows): the panel moves between HBM and the
  // registers through a wave-private LDS stage, 16 rows x 64 B per memory instruction (four lanes
  // per row) instead of 64 rows x 16 B: a row-per-lane access touches 64 cache lines per
  // instruction with half of each used, and the load + store of the panel alone took 94 of the
  // 116 us of a 1472-row launch (tools/lupanelbench.hip, profiles/r04_lupanelbench.txt).  Rows come
  // in by LDS-DMA (no staging registers), two 64-row blocks per wave in flight; in the stage, the
  // 16-B chunk c of block row r sits at position c ^ ((r >> 2) & 3) (conflict-free row reads).
  constexpr bool STAGED = NT == 256 && NB == 16;
  __shared__ __attribute__((aligned(16))) float pst[STAGED ? NWV : 1][2][STAGED ? 64 * kNB : 1];
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const f4v lds_cf4;
  typedef __attribute__((address_space(3))) f4v lds_f4;
  const bool staged = STAGED && vec;
  // rows >= R read as zero (every use below is masked); the range ends at the panel's last row
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(Ab + (size_t)k0 * N + k0, 0, ((R - 1) * N + kNB) * 4, 0x00020000);
  static_assert(!FUSE || (NT == 256 && NB == 16), "FUSE: staged 16-wide panels only");
  static_assert(JQ >= 0 && JQ <= 3 && (FUSE || JQ == 0), "JQ: earlier panels of the half (FUSE)");
  __shared__ float Ut[FUSE ? kNB : 1][FUSE ? 3 * kNB : 1];
  if (staged) {
    // lane l of instruction i of block m: block row 16 i + (l >> 2), stage position l & 3, source
    // chunk (l & 3) ^ ((l >> 4) & 3)
    const unsigned vo = (unsigned)(((wave * 64 + (lane >> 2)) * N + 4 * ((lane & 3) ^ ((lane >> 4) & 3))) * 4);
    auto issue = [&](int m) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, (lds_void*)(&pst[wave][m & 1][i * 256]), 16, vo,
                                                 (kLuThreads * m + 16 * i) * N * 4, 0, 0);
    };
    const unsigned rb = (unsigned)(uintptr_t)(lds_cf4*)(const f4v*)&pst[wave][0][lane * kNB];
    const int sr = (lane >> 2) & 3;
    if constexpr (FUSE && JQ > 0) {
      // the JQ earlier panels' U rows on this panel's columns to LDS; per 64-row block, this block's A
      // rows into stage buffer 0 and, one earlier panel at a time, the same rows' L into buffer 1 (one
      // block in flight: the panels are not bound by their load latency,
      // profiles/r06_lu_ab_panel_asm_reads_rejected.txt)
      __shared__ __attribute__((aligned(16))) float Uq[JQ * kNB][kNB];
      for (int e = tid; e < JQ * kNB * kNB; e += kLuThreads)
        Uq[e >> 4][e & 15] = Ab[(size_t)(k0 - JQ * kNB + (e >> 4)) * N + k0 + (e & 15)];
      __syncthreads();
#pragma unroll
      for (int m = 0; m < M; ++m) {
        // rows [k0, cend) (m = 0, tid < cend - k0) already carry every earlier panel's update (slab):
        // their lanes multiply by l = 0 (-0 * u adds nothing); the stage traffic is whole-wave
        const bool upd = m > 0 || k0 + tid >= cend;
#pragma unroll
        for (int q = 0; q < JQ; ++q) {
          const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
              Ab + (size_t)k0 * N + k0 - (JQ - q) * kNB, 0, ((R - 1) * N + kNB) * 4, 0x00020000);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (q == 0)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, (lds_void*)(&pst[wave][0][i * 256]), 16, vo,
                                                       (kLuThreads * m + 16 * i) * N * 4, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, (lds_void*)(&pst[wave][1][i * 256]), 16, vo,
                                                     (kLuThreads * m + 16 * i) * N * 4, 0, 0);
          }
          vm_wait<0>();
          if (q == 0) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const f4v v = *(lds_cf4*)(uintptr_t)(rb + (unsigned)(((c ^ sr) * 4) * 4));
              a[m][4 * c] = v.x; a[m][4 * c + 1] = v.y; a[m][4 * c + 2] = v.z; a[m][4 * c + 3] = v.w;
            }
          }
          const unsigned lb = rb + (unsigned)(64 * kNB * 4);
#pragma unroll
          for (int g = 0; g < 4; ++g) {  // L[row][k0 - 16 (JQ - q) + 4 g .. + 4)
            const f4v lq = *(lds_cf4*)(uintptr_t)(lb + (unsigned)(((g ^ sr) * 4) * 4));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lv = upd ? (e == 0 ? lq.x : (e == 1 ? lq.y : (e == 2 ? lq.z : lq.w))) : 0.f;
              const int li = q * kNB + 4 * g + e;
#pragma unroll
              for (int c4 = 0; c4 < 4; ++c4) {
                const f4v u = *reinterpret_cast<const f4v*>(&Uq[li][4 * c4]);
                // (U is the same for every lane: scalar operands, so the unrolled sections do not hold
                // their U values in vector registers -- with them, JQ = 2 spilled 240 B per lane)
                const float u0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(u.x)));
                const float u1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(u.y)));
                const float u2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(u.z)));
                const float u3 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(u.w)));
                a[m][4 * c4] = fmaf(-lv, u0, a[m][4 * c4]);
                a[m][4 * c4 + 1] = fmaf(-lv, u1, a[m][4 * c4 + 1]);
                a[m][4 * c4 + 2] = fmaf(-lv, u2, a[m][4 * c4 + 2]);
                a[m][4 * c4 + 3] = fmaf(-lv, u3, a[m][4 * c4 + 3]);
              }
            }
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): both buffers read before they refill
          __builtin_amdgcn_sched_barrier(0);   // (each earlier panel's share in its own scheduling region)
        }
      }
    } else {
    issue(0);
    if (M > 1) issue(1);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m + 1 < M) vm_wait<4>(); else vm_wait<0>();  // block m landed (block m + 1 may be in flight)
      const unsigned ra = rb + (unsigned)((m & 1) * 64 * kNB * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f4v v = *(lds_cf4*)(uintptr_t)(ra + (unsigned)(((c ^ sr) * 4) * 4));
        a[m][4 * c] = v.x; a[m][4 * c + 1] = v.y; a[m][4 * c + 2] = v.z; a[m][4 * c + 3] = v.w;
      }
      if (m + 2 < M) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this buffer's reads done before it refills
        issue(m + 2);
      }
    }
    }
  } else {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int r = tid + kLuThreads * m;
      const float* src = Ab + (size_t)(k0 + min(r, R - 1)) * N + k0;
      if (vec) {
#pragma unroll
        for (int c4 = 0; c4 < kNB; c4 += 4) {
          const float4 v = *reinterpret_cast<const float4*>(src + c4);
          a[m][c4] = v.x; a[m][c4 + 1] = v.y; a[m][c4 + 2] = v.z; a[m][c4 + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int c = 0; c < kNB; ++c) a[m][c] = src[min(c, nb - 1)];
      }
      // (no zero fill of rows >= R / columns >= nb: every use below is masked, and overwriting a
      // register a load is still filling would stall on that load right here)
    }
  }

  if constexpr (DIAG & 1) {
    if (tid < kNB) pvs[tid] = k0 + tid;
  }
#pragma unroll
  for (int j = 0; j < kNB; ++j) {
    if (!(DIAG & 1) && j < nb) {
      const int q = j & 1;
      float best = -1.f;
      int bi = R;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int r = tid + kLuThreads * m;
        const float v = fabsf(col_of(a[m], j));
        if (r >= j && r < R && v > best) { best = v; bi = r; }
      }
      wave_argmax(best, bi);
      // the wave's winner (a row of one of its own lanes) publishes its whole row, so no second
      // round trip is needed once the waves' winners are compared
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (tid + kLuThreads * m == bi) {
#pragma unroll
          for (int c = 0; c < kNB; ++c) cand[q][wave][c] = a[m][c];
        }
      if (lane == 0) { rv[q][wave] = best; ri[q][wave] = bi; }
      if (tid == j) {
#pragma unroll
        for (int c = 0; c < kNB; ++c) rowj[q][c] = a[0][c];
      }
      __syncthreads();
      // every thread combines the waves' winners (same order and tie rule as the shuffle tree)
      float bv = rv[q][0];
      int bx = ri[q][0], bw = 0;
#pragma unroll
      for (int w = 1; w < NWV; ++w) {
        const float ov = rv[q][w];
        const int oi = ri[q][w];
        if (ov > bv || (ov == bv && oi < bx)) { bv = ov; bx = oi; bw = w; }
      }
      const bool nan_col = bx >= R;  // all entries NaN: keep the diagonal
      const int p = nan_col ? j : bx;
      if (tid == 0) {
        if (!nan_col && bv == 0.f && info[b] == 0) info[b] = k0 + j + 1;
        piv[b * N + k0 + j] = k0 + p + 1;
        pvs[j] = k0 + p;
      }
      float pr[kNB];
#pragma unroll
      for (int c = 0; c < kNB; ++c) pr[c] = nan_col ? rowj[q][c] : cand[q][bw][c];
      // the owner of row p takes row j's values, the owner of row j the pivot row
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (tid + kLuThreads * m == p) {
#pragma unroll
          for (int c = 0; c < kNB; ++c) a[m][c] = rowj[q][c];
        }
      if (tid == j) {
#pragma unroll
        for (int c = 0; c < kNB; ++c) a[0][c] = pr[c];
      }
      const float pv = pr[j];
      if (pv != 0.f) {
        const float rcp = 1.0f / pv;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = tid + kLuThreads * m;
          if (r > j && r < R) {
            const float l = col_of(a[m], j) * rcp;
#pragma unroll
            for (int c = 0; c < kNB; ++c) {  // static register indices: j is not a compile-time constant
              if (c == j) a[m][c] = l;
              else if (c > j) a[m][c] = fmaf(-l, pr[c], a[m][c]);
            }
          }
        }
      }
    }
  }

  // write the factored panel back; L11 for the in-block substitution
  if (staged) {  // through the stage: own row in, 16 rows x 64 B out per store instruction
    const unsigned wb = (unsigned)(uintptr_t)(lds_f4*)(f4v*)&pst[wave][0][0];
    const int sr = (lane >> 2) & 3;
    const unsigned vo = (unsigned)(((wave * 64 + (lane >> 2)) * N + 4 * ((lane & 3) ^ ((lane >> 4) & 3))) * 4);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const unsigned bb = wb + (unsigned)((m & 1) * 64 * kNB * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        *(lds_f4*)(uintptr_t)(bb + (unsigned)((lane * kNB + (c ^ sr) * 4) * 4)) =
            f4v{a[m][4 * c], a[m][4 * c + 1], a[m][4 * c + 2], a[m][4 * c + 3]};
      f4v o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = *(lds_cf4*)(uintptr_t)(bb + (unsigned)((i * 256 + lane * 4) * 4));
      // every value in registers before the first store, and the stores drained before the next
      // block's LDS reads: an LDS return into the registers of a store still in flight made the
      // factors nondeterministic (the compiler reuses them; profiles/r04_lupanelbench_staged.txt).
      // Draining costs nothing measurable (same file: 121-123 vs 126-129 us at 1984 rows).
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o[i]), prs, vo, (kLuThreads * m + 16 * i) * N * 4, 0);
      vm_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int r = tid + kLuThreads * m;
    if (!staged && r < R) {
      float* dst = Ab + (size_t)(k0 + r) * N + k0;
      if (vec) {
#pragma unroll
        for (int c4 = 0; c4 < kNB; c4 += 4)
          *reinterpret_cast<float4*>(dst + c4) = make_float4(a[m][c4], a[m][c4 + 1], a[m][c4 + 2], a[m][c4 + 3]);
      } else {
#pragma unroll
        for (int c = 0; c < kNB; ++c)
          if (c < nb) dst[c] = a[m][c];
      }
    }
  }
  if (tid < nb) {
#pragma unroll
    for (int c = 0; c < kNB; ++c) L11[tid][c] = a[0][c];
  }
  if constexpr (FUSE) {
    // U rows of this panel on the half's later columns (panel_finish, also to Ut), then the slab
    // update: the later panels' rows [k0 + 16, cend) -= L U, by the threads holding those rows' L (m = 0)
    const bool slab = k0 + kNB < cend;
    panel_finish<kNB>(Ab, N, K0, k0, nb, cend, L11, pvs, prow, pcur, pcnt, slab ? Ut : nullptr);
    if (slab) {
      __syncthreads();
      const int W = cend - k0 - kNB;  // 16, 32 or 48 (a full half)
      if (tid >= kNB && tid < cend - k0) {
        float* row = Ab + (size_t)(k0 + tid) * N + k0 + kNB;
        // this row's L as the write-back above stored it (re-read: keeping a[0] live through
        // panel_finish cost the small panels registers)
        float lr[kNB];
#pragma unroll
        for (int c4 = 0; c4 < kNB / 4; ++c4) {
          const float4 t = *reinterpret_cast<const float4*>(row - kNB + 4 * c4);
          lr[4 * c4] = t.x; lr[4 * c4 + 1] = t.y; lr[4 * c4 + 2] = t.z; lr[4 * c4 + 3] = t.w;
        }
#pragma unroll 1
        for (int c4 = 0; c4 < W / 4; ++c4) {
          float4 v = *reinterpret_cast<const float4*>(row + 4 * c4);
#pragma unroll
          for (int li = 0; li < kNB; ++li) {
            const float lv = lr[li];
            v.x = fmaf(-lv, Ut[li][4 * c4], v.x);
            v.y = fmaf(-lv, Ut[li][4 * c4 + 1], v.y);
            v.z = fmaf(-lv, Ut[li][4 * c4 + 2], v.z);
            v.w = fmaf(-lv, Ut[li][4 * c4 + 3], v.w);
          }
          *reinterpret_cast<float4*>(row + 4 * c4) = v;
        }
      }
    }
  } else if constexpr (!(DIAG & 2)) {
    panel_finish<kNB>(Ab, N, K0, k0, nb, cend, L11, pvs, prow, pcur, pcnt);
  }
}

// Global-memory panel for N > 10240 (rows beyond what the register panel can hold, up to the
// solve's N <= 36736): the same column steps as lu_panel_kernel with the NB-wide panel in HBM /
// L2 instead of registers (thread t owns rows k0 + t + NT i); the pivot row exchange and the
// rank-1 update read and write the panel in place, a workgroup-wide barrier between the steps.
// Same pivot rule (first max |a|) and operation order per element as the register panel.
template <int NB, int NT>
__global__ __launch_bounds__(NT, 1) void lu_panel_global_kernel(int N, int K0, int k0, int cend, float* A, int* piv,
                                                                int* info) {
  constexpr int NWV = NT / 64;
  __shared__ float prw[NB];
  __shared__ float L11[NB][NB + 1];
  __shared__ float rv[NWV];
  __shared__ int ri[NWV + 1];
  __shared__ int pvs[NB], prow[2 * NB], pcur[2 * NB], pcnt[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  const int nb = min(NB, min(N - k0, cend - k0));
  for (int j = 0; j < nb; ++j) {
    const int c = k0 + j;
    float best = -1.f;
    int bi = N;
    for (int r = c + tid; r < N; r += NT) {
      const float v = fabsf(Ab[(size_t)r * N + c]);
      if (v > best) { best = v; bi = r; }
    }
    wave_argmax(best, bi);
    if (lane == 0) { rv[wave] = best; ri[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float bv = rv[0];
      int bx = ri[0];
      for (int w = 1; w < NWV; ++w)
        if (rv[w] > bv || (rv[w] == bv && ri[w] < bx)) { bv = rv[w]; bx = ri[w]; }
      if (bx >= N) bx = c;  // all entries NaN: keep the diagonal
      else if (bv == 0.f && info[b] == 0) info[b] = c + 1;
      ri[NWV] = bx;
      piv[b * N + c] = bx + 1;
      pvs[j] = bx;
    }
    __syncthreads();
    const int p = ri[NWV];
    if (tid < nb) {  // exchange rows c and p on the panel's columns; the pivot row to LDS
      float* rc = Ab + (size_t)c * N + k0 + tid;
      float* rp = Ab + (size_t)p * N + k0 + tid;
      const float vc = *rc, vp = *rp;
      if (p != c) { *rc = vp; *rp = vc; }
      prw[tid] = vp;
    }
    __syncthreads();
    const float pv = prw[j];
    if (pv != 0.f) {
      const float rcp = 1.0f / pv;
      for (int r = c + 1 + tid; r < N; r += NT) {
        float* row = Ab + (size_t)r * N + k0;
        const float l = row[j] * rcp;
        row[j] = l;
        for (int cc = j + 1; cc < nb; ++cc) row[cc] = fmaf(-l, prw[cc], row[cc]);
      }
    }
    __syncthreads();  // the next column's search reads the updated panel; prw is rewritten
  }
  if (tid < nb) {
    for (int cc = 0; cc < NB; ++cc) L11[tid][cc] = cc < nb ? Ab[(size_t)(k0 + tid) * N + k0 + cc] : 0.f;
  }
  panel_finish<NB>(Ab, N, K0, k0, nb, cend, L11, pvs, prow, pcur, pcnt);
}

// A[c0.., c0..cend) -= L21 U12 inside the current 64-column half, c0 = k0 + NB: rows
// [c0 + blockIdx.y*64, +64) of instance blockIdx.x, w = cend - c0 <= 64 - NB columns.  Every thread
// issues all of its loads (U12 and L21 pieces, then its A elements) at once from clamped, valid
// addresses before it uses any: a fixed count per thread, no loop-carried load -> use -> load chain.
template <int NB>
__global__ __launch_bounds__(256) void lu_update_block_kernel(int N, int k0, int cend, float* A) {
  constexpr int kW = kBlk - NB;                       // widest update
  constexpr int kUq = (NB * kW + 255) / 256;          // U12 elements per thread
  constexpr int kLq = (kUpdRows * NB + 255) / 256;    // L21 elements per thread
  constexpr int kAq = (kUpdRows * kW + 255) / 256;    // A elements per thread
  __shared__ float Us[NB][kW];
  __shared__ float Ls[kUpdRows][NB + 1];
  const int tid = threadIdx.x;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = k0 + NB, w = cend - c0;
  const int r0 = c0 + blockIdx.y * kUpdRows;
  const int rows = min(kUpdRows, N - r0);
  if (rows <= 0 || w <= 0) return;
  float u[kUq], l[kLq], a[kAq];
#pragma unroll
  for (int q = 0; q < kUq; ++q) {
    const int idx = min(tid + 256 * q, NB * kW - 1), li = idx / kW, c = min(idx % kW, w - 1);
    u[q] = Ab[(size_t)(k0 + li) * N + c0 + c];
  }
#pragma unroll
  for (int q = 0; q < kLq; ++q) {
    const int idx = min(tid + 256 * q, kUpdRows * NB - 1), r = min(idx / NB, rows - 1), li = idx % NB;
    l[q] = Ab[(size_t)(r0 + r) * N + k0 + li];
  }
#pragma unroll
  for (int q = 0; q < kAq; ++q) {
    const int idx = min(tid + 256 * q, kUpdRows * kW - 1), r = min(idx / kW, rows - 1), c = min(idx % kW, w - 1);
    a[q] = Ab[(size_t)(r0 + r) * N + c0 + c];
  }
#pragma unroll
  for (int q = 0; q < kUq; ++q) {
    const int idx = tid + 256 * q;
    if (idx < NB * kW) Us[idx / kW][idx % kW] = u[q];
  }
#pragma unroll
  for (int q = 0; q < kLq; ++q) {
    const int idx = tid + 256 * q;
    if (idx < kUpdRows * NB) Ls[idx / NB][idx % NB] = l[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kAq; ++q) {
    const int idx = tid + 256 * q, r = idx / kW, c = idx % kW;
    if (idx < kUpdRows * kW && r < rows && c < w) {
      float v = a[q];
#pragma unroll
      for (int li = 0; li < NB; ++li) v = fmaf(-Ls[r][li], Us[li][c], v);
      Ab[(size_t)(r0 + r) * N + c0 + c] = v;
    }
  }
}

// The same update when the half's remaining width is exactly W (a multiple of 16; N % 4 == 0 and
// 16-B aligned rows): 16-B accesses, and only as many threads per row as the width needs (the
// generic kernel sizes every launch for the widest update and clamps the rest onto repeated
// loads).  Same operations in the same order per element as lu_update_block_kernel.
template <int NB, int W>
__global__ __launch_bounds__(256) void lu_update_block_vec_kernel(int N, int k0, float* A) {
  constexpr int kW4 = W / 4, kNB4 = NB / 4;
  constexpr int kAq = kUpdRows * kW4 / 256;              // float4 of A per thread
  constexpr int kUq = (NB * kW4 + 255) / 256;             // float4 of U12 per thread
  constexpr int kLq = (kUpdRows * kNB4 + 255) / 256;      // float4 of L21 per thread
  static_assert(kAq * 256 == kUpdRows * kW4, "W must be a multiple of 16");
  __shared__ __attribute__((aligned(16))) float Us[NB][W];
  __shared__ float Ls[kUpdRows][NB + 1];
  const int tid = threadIdx.x;
  float* Ab = A + blockIdx.x * (size_t)N * N;
  const int c0 = k0 + NB;
  const int r0 = c0 + blockIdx.y * kUpdRows;
  const int rows = min(kUpdRows, N - r0);
  float4 u[kUq], l[kLq], a[kAq];
#pragma unroll
  for (int q = 0; q < kUq; ++q) {
    const int idx = min(tid + 256 * q, NB * kW4 - 1), li = idx / kW4, c = (idx % kW4) * 4;
    u[q] = *reinterpret_cast<const float4*>(Ab + (size_t)(k0 + li) * N + c0 + c);
  }
#pragma unroll
  for (int q = 0; q < kLq; ++q) {
    const int idx = min(tid + 256 * q, kUpdRows * kNB4 - 1), r = min(idx / kNB4, rows - 1), li = (idx % kNB4) * 4;
    l[q] = *reinterpret_cast<const float4*>(Ab + (size_t)(r0 + r) * N + k0 + li);
  }
#pragma unroll
  for (int q = 0; q < kAq; ++q) {
    const int idx = tid + 256 * q, r = min(idx / kW4, rows - 1), c = (idx % kW4) * 4;
    a[q] = *reinterpret_cast<const float4*>(Ab + (size_t)(r0 + r) * N + c0 + c);
  }
#pragma unroll
  for (int q = 0; q < kUq; ++q) {
    const int idx = tid + 256 * q;
    if (idx < NB * kW4) *reinterpret_cast<float4*>(&Us[idx / kW4][(idx % kW4) * 4]) = u[q];
  }
#pragma unroll
  for (int q = 0; q < kLq; ++q) {
    const int idx = tid + 256 * q;
    if (idx < kUpdRows * kNB4) {
      float* d = &Ls[idx / kNB4][(idx % kNB4) * 4];
      d[0] = l[q].x; d[1] = l[q].y; d[2] = l[q].z; d[3] = l[q].w;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kAq; ++q) {
    const int idx = tid + 256 * q, r = idx / kW4, c = (idx % kW4) * 4;
    if (r < rows) {
      float4 v = a[q];
#pragma unroll
      for (int li = 0; li < NB; ++li) {
        const float lv = Ls[r][li];
        const float4 uv = *reinterpret_cast<const float4*>(&Us[li][c]);
        v.x = fmaf(-lv, uv.x, v.x); v.y = fmaf(-lv, uv.y, v.y); v.z = fmaf(-lv, uv.z, v.z); v.w = fmaf(-lv, uv.w, v.w);
      }
      *reinterpret_cast<float4*>(Ab + (size_t)(r0 + r) * N + c0 + c) = v;
    }
  }
}

// In-half update after the panel at k0 (rank NB on the half's columns [k0 + NB, cend)).
template <int NB>
static void lu_update_block(int64_t B, int64_t N, int k0, int cend, float* A, bool vec, hipStream_t s) {
  const int c0 = k0 + NB, w = cend - c0;
  const dim3 grid((unsigned)B, (unsigned)((N - c0 + kUpdRows - 1) / kUpdRows));
  if (vec && w == 48) hipLaunchKernelGGL((lu_update_block_vec_kernel<NB, 48>), grid, dim3(256), 0, s, (int)N, k0, A);
  else if (vec && w == 32) hipLaunchKernelGGL((lu_update_block_vec_kernel<NB, 32>), grid, dim3(256), 0, s, (int)N, k0, A);
  else if (vec && w == 16) hipLaunchKernelGGL((lu_update_block_vec_kernel<NB, 16>), grid, dim3(256), 0, s, (int)N, k0, A);
  else hipLaunchKernelGGL(lu_update_block_kernel<NB>, grid, dim3(256), 0, s, (int)N, k0, cend, A);
}

// The net row permutation of the interchanges of rows [K0, cend) (a 64-column half or, composed, a
// whole 128-column block: nbk <= 128), one wave per instance, into perm[b] = {rowid[256], cur[256],
// cnt} (kPermInts ints).
constexpr int kPermMax = 128;
constexpr int kPermInts = 4 * kPermMax + 1;
__global__ __launch_bounds__(64) void lu_block_perm_kernel(int N, int K0, int cend, const int* piv, int* perm) {
  __shared__ int pvs[kPermMax], prow[2 * kPermMax], pcur[2 * kPermMax], pcnt[1];
  const int tid = threadIdx.x, nbk = cend - K0;
  const size_t b = blockIdx.x;
  for (int i = tid; i < nbk; i += 64) pvs[i] = piv[b * N + K0 + i] - 1;
  __syncthreads();
  build_row_perm(pvs, K0, nbk, prow, pcur, pcnt);
  int* out = perm + b * kPermInts;
  for (int i = tid; i < 2 * kPermMax; i += 64) { out[i] = prow[i]; out[2 * kPermMax + i] = pcur[i]; }
  if (tid == 0) out[4 * kPermMax] = *pcnt;
}

// The row interchanges of rows [K0, K0 + nbk) (perm from lu_block_perm_kernel, nbk <= NBK) on the
// columns [a0, a1) and [b0, b1) (one thread per column), and for the columns [b0, trsm_end) (TRSM:
// NBK == nbk == 64) U12 = L11^-1 A12 on the block rows (L11 = the block's unit-lower multipliers, in
// LDS, broadcast reads).  Every row outside the block that the interchanges touch ends up holding
// an original block row, so: the new block rows are loaded first (x, registers), then the outside
// rows are moved 16 at a time (their sources are block rows, which are only stored to afterwards),
// then the substitution and the block-row stores.
// BUILD (one workgroup per instance, r04): the permutation is built here from piv by wave 0
// (build_row_perm) instead of read from perm -- no lu_block_perm_kernel launch in front.
template <int NBK, bool TRSM, bool BUILD = false>
__global__ __launch_bounds__(256) void lu_swap_kernel(int N, int K0, int nbk, int a0, int a1, int b0, int b1,
                                                      int trsm_end, float* A, const int* perm, const int* piv) {
  __shared__ float Ld[TRSM ? kBlk : 1][kBlk + 1];
  __shared__ int prow[2 * kPermMax], pcur[2 * kPermMax], pcnt[1];
  __shared__ int pvs[BUILD ? kPermMax : 1];
  const int tid = threadIdx.x;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  if constexpr (TRSM) {  // (256 threads: the 64 x 64 block's 16 loads per thread all in flight at once)
    constexpr int kLq = kBlk * kBlk / 256;
    float lv[kLq];
#pragma unroll
    for (int q = 0; q < kLq; ++q) {
      const int idx = tid + 256 * q, r = idx / kBlk, c = idx % kBlk;
      lv[q] = Ab[(size_t)(K0 + r) * N + K0 + c];
    }
#pragma unroll
    for (int q = 0; q < kLq; ++q) {
      const int idx = tid + 256 * q;
      Ld[idx / kBlk][idx % kBlk] = lv[q];
    }
  }
  if constexpr (BUILD) {
    for (int i = tid; i < nbk; i += blockDim.x) pvs[i] = piv[b * N + K0 + i] - 1;
    __syncthreads();
    build_row_perm(pvs, K0, nbk, prow, pcur, pcnt);  // (ends with a barrier)
  } else {
    const int* pb = perm + b * kPermInts;
    for (int i = tid; i < 2 * kPermMax; i += blockDim.x) { prow[i] = pb[i]; pcur[i] = pb[2 * kPermMax + i]; }
    if (tid == 0) *pcnt = pb[4 * kPermMax];
    __syncthreads();
  }
  const int cnt = *pcnt;
  const int q = blockIdx.y * blockDim.x + tid, na = a1 - a0;
  const int c = q < na ? a0 + q : b0 + (q - na);
  if (q >= na && c >= b1) return;
  // (all loads unconditional, from valid rows: a conditional load makes the compiler drain every
  // outstanding load at its use, serialising the column's moves)
  float x[NBK];
#pragma unroll
  for (int i = 0; i < NBK; ++i) x[i] = Ab[(size_t)pcur[min(i, nbk - 1)] * N + c];
  for (int i0 = nbk; i0 < cnt; i0 += 16) {
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = Ab[(size_t)pcur[min(i0 + i, cnt - 1)] * N + c];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i0 + i < cnt) Ab[(size_t)prow[i0 + i] * N + c] = y[i];
  }
  if constexpr (TRSM) {
    if (q >= na && c < trsm_end) {
#pragma unroll
      for (int i = 1; i < kBlk; ++i) {
        float s = x[i];
#pragma unroll
        for (int l = 0; l < i; ++l) s = fmaf(-Ld[i][l], x[l], s);
        x[i] = s;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NBK; ++i)
    if (i < nbk) Ab[(size_t)(K0 + i) * N + c] = x[i];
}

// A22 -= L21 U12 (rank 64) on the trailing matrix [c0, N) x [c0, cmax), c0 = K0 + 64 (cmax = N, or
// K0 + 128 for the second half of a 128-column block: the "mid" update of lu_factor_blocks).  A workgroup (8 waves,
// one per CU) owns a 128-column strip [cb, cb + 128) over kTRW rows [rs, re): U12's 64 x 128
// block is staged once, transposed, in LDS (Ut); the rows are streamed in steps of 64 with a
// one-step software pipeline.  A22 moves between HBM and the accumulators through LDS (Cin /
// Cout) so that the global accesses are row-contiguous 16-B lanes (512 B per row per half-wave:
// the MFMA layout's own 2-rows-x-128-B dword pattern ran at a third of that rate); -L21 is
// staged in LDS (Ls).  Wave (wr, wc) owns 32 x 32 of a step = one
// v_mfma_f32_32x32x2f32 accumulator; both operands are 16-B LDS reads along k: lane half h covers
// k in [32h, 32h + 32) and MFMA step s uses k = 32h + s (any k order gives the same sum set).  The
// strips of one instance are consecutive logical ids on one XCD (its L2 serves the -L21 re-reads
// of the 16 strips).  VEC: N % 4 == 0 and 16-B aligned rows (16-B global accesses).
// DIAG (tools/lubench.hip only): 1 = no MFMAs (the memory pipeline alone).
// TCW = 64 (the mid update, whose strip is the block's second half only): the loads, stores and
// U12 staging cover 64 columns and the waves of columns 64..127 skip their MFMAs (r03: the full
// 128-column mapping loaded and zero-masked the other half, twice the A22 reads).
template <bool VEC, int DIAG = 0, int TCW = kTC>
__global__ __launch_bounds__(kTrailThreads, 1) void lu_trail_kernel(int N, int K0, int ntc, int nrc, int cmax,
                                                                      float* A) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int kCSw = TCW + 8;         // A22 tile stride (8 mod 32 banks: conflict-free acc access)
  float* Ut = sm;                       // [TCW cols][kTS]: U12^T
  float* Lsb = Ut + TCW * kTS;          // [kTRS rows][kTS]: -L21
  float* Cin = Lsb + kTRS * kTS;        // [kTRS rows][kCSw]: next step's A22 rows
  float* Cout = Cin + kTRS * kCSw;      // [kTRS rows][kCSw]: this step's result rows
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int per = ntc * nrc;
  const size_t b = (size_t)(logical / per);
  const int t = logical % per, rc = t / ntc, tc = t % ntc;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = K0 + kBlk;
  const int cb = c0 + tc * kTC, rs = c0 + rc * kTRW, re = min(N, rs + kTRW);
  const int nsteps = (re - rs + kTRS - 1) / kTRS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, il = lane & 31, h = lane >> 5;
  const int wr = (wave >> 2) * 32, wc = (wave & 3) * 32;
  constexpr int NT = kTrailThreads;

  typedef typename std::conditional<VEC, float4, float>::type VT;
  constexpr int W = VEC ? 4 : 1;                    // floats per global access
  constexpr int kCQ = kTRS * TCW / W / NT;          // A22 accesses per thread per step
  constexpr int kLQ = kTRS * kBlk / W / NT;         // -L21 accesses per thread per step
  constexpr int kUQ = kBlk * TCW / W / NT;          // U12 accesses per thread
  constexpr int CPR = TCW / W, LPR = kBlk / W;      // accesses per row
  auto ld = [&](int row, int col, bool ok) -> VT {  // clamped address, masked value
    const float* p = Ab + (size_t)row * N + col;
    if constexpr (VEC) {
      const float4 x = *reinterpret_cast<const float4*>(p);
      return ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const float x = *p;
      return ok ? x : 0.f;
    }
  };
  auto st_lds = [&](float* d, const VT& v, float sgn) {
    if constexpr (VEC) *reinterpret_cast<float4*>(d) = make_float4(sgn * v.x, sgn * v.y, sgn * v.z, sgn * v.w);
    else *d = sgn * v;
  };
  auto loadC = [&](int step, VT (&c)[kCQ]) {
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, row = rs + step * kTRS + e / CPR, col = cb + (e % CPR) * W;
      c[q] = ld(min(row, re - 1), min(col, N - W), row < re && col < cmax);
    }
  };
  auto loadL = [&](int step, VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q, row = rs + step * kTRS + e / LPR;
      l[q] = ld(min(row, re - 1), K0 + (e % LPR) * W, row < re);
    }
  };
  auto writeC = [&](const VT (&c)[kCQ]) {
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q;
      st_lds(Cin + (e / CPR) * kCSw + (e % CPR) * W, c[q], 1.f);
    }
  };
  auto writeL = [&](const VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q;
      st_lds(Lsb + (e / LPR) * kTS + (e % LPR) * W, l[q], -1.f);
    }
  };
  auto storeOut = [&](int step) {
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, row = rs + step * kTRS + e / CPR, col = cb + (e % CPR) * W;
      if (row < re && col < cmax) {
        const float* s = Cout + (e / CPR) * kCSw + (e % CPR) * W;
        if constexpr (VEC) *reinterpret_cast<float4*>(Ab + (size_t)row * N + col) = *reinterpret_cast<const float4*>(s);
        else Ab[(size_t)row * N + col] = *s;
      }
    }
  };
  // accumulator register v <-> tile row wr + 8(v/4) + 4h + v%4, column wc + il (waves of columns
  // >= TCW have no tile)
  const bool tile = TCW == kTC || wc < TCW;
  auto accFromCin = [&](floatx16& acc) {
    if (!tile) return;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = Cin[(wr + 8 * (v >> 2) + 4 * h + (v & 3)) * kCSw + wc + il];
  };
  auto accToCout = [&](const floatx16& acc) {
    if (!tile) return;
#pragma unroll
    for (int v = 0; v < 16; ++v) Cout[(wr + 8 * (v >> 2) + 4 * h + (v & 3)) * kCSw + wc + il] = acc[v];
  };

  VT cr[kCQ], lr[kLQ];
  loadC(0, cr);
  loadL(0, lr);
#pragma unroll
  for (int q = 0; q < kUQ; ++q) {  // U12 block -> Ut (transposed)
    const int e = tid + NT * q, k = e / CPR, cl = (e % CPR) * W, col = cb + cl;
    const VT u = ld(K0 + k, min(col, N - W), col < cmax);
    if constexpr (VEC) {
      Ut[(cl + 0) * kTS + k] = u.x; Ut[(cl + 1) * kTS + k] = u.y;
      Ut[(cl + 2) * kTS + k] = u.z; Ut[(cl + 3) * kTS + k] = u.w;
    } else {
      Ut[cl * kTS + k] = u;
    }
  }
  writeC(cr);
  writeL(lr);
  __syncthreads();
  floatx16 acc = {};
  accFromCin(acc);

  for (int step = 0; step < nsteps; ++step) {
    const bool more = step + 1 < nsteps;
    if (more) {
      loadC(step + 1, cr);
      loadL(step + 1, lr);
    }
    if (DIAG != 1 && tile) {
      const float* Ls = Lsb;
#pragma unroll
      for (int sg = 0; sg < 8; ++sg) {
        const float4 fa = *reinterpret_cast<const float4*>(Ls + (wr + il) * kTS + 32 * h + 4 * sg);
        const float4 fb = *reinterpret_cast<const float4*>(Ut + (wc + il) * kTS + 32 * h + 4 * sg);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(fb, s4), acc, 0, 0, 0);
      }
    }
    accToCout(acc);
    __syncthreads();  // Cin (this step's rows) and Ls fully consumed, Cout complete
    if (more) {
      writeC(cr);
      writeL(lr);
    }
    storeOut(step);
    __syncthreads();  // Cout drained, Cin / Ls hold the next step
    if (more) accFromCin(acc);
  }
}

// ------------------------------------------------------------------------------------------------
// 128-column outer blocks (r03).  The rank-64 update streams A22 through HBM once per 64 columns at
// 16 flop/B, under the fp32 MFMA ridge; per 128-column block [P, P + 128) the two 64-column halves
// are factored one after the other (the second half updated by the first: the rank-64 "mid" update
// of lu_trail_kernel restricted to [P + 64, P + 128)), and the rest of the matrix gets ONE rank-128
// update: half the A22 traffic, 32 flop/B.  U12 = L11^-1 A12 for the 128 block rows is a two-level
// MFMA substitution with the inverted 32 x 32 diagonal blocks of L11 (lu_linv_kernel, r05), fused into
// the trailing update's prologue (every strip's workgroup owns its 128 columns of A12 and A22, so no other
// workgroup reads what it overwrites).
constexpr int kOB = 2 * kBlk;     // outer block width = rank of the fused trailing update
constexpr int kT2C = 128;         // trailing update: columns per workgroup strip
constexpr int kT2S = 32;          //   rows per pipeline step
constexpr int kT2K = kOB + 4;     //   LDS stride (k) of the U12^T and L21 tiles
constexpr int kT2CS = kT2C + 8;   //   LDS stride of the product tile
constexpr int kT2LK = kOB + 4;    //   LDS stride of the prologue's staged two-level L11^-1
constexpr int kT2Threads = 256;   // 4 waves; two workgroups per CU
// the block's composed row permutation for the gathered loads: the block rows' sources, the displaced
// rows below the block with their sources (as given, then sorted by row), a bitmap of the displaced
// rows (one word per step) and the rank of each step's first displaced row (one byte per step)
constexpr int kT2BitWords = (kLuMaxN + kT2S - 1) / kT2S + 2;
// L21 and the product tile double-buffered; the prologue's half tiles and U12^T over them
constexpr int kT2MainFloats = 2 * kT2S * kT2K + 2 * kT2S * kT2CS;
constexpr int kT2ProFloats = kOB * kT2LK;
constexpr int kT2AreaFloats = kT2MainFloats > kT2ProFloats ? kT2MainFloats : kT2ProFloats;
constexpr size_t kT2Lds = (size_t)kT2AreaFloats * sizeof(float) + (size_t)(4 * kPermMax + kT2BitWords) * sizeof(int) +
                          (size_t)((kT2BitWords + 3) & ~3);
static_assert(kT2C * kT2K <= kT2AreaFloats, "U12^T staging must fit the area");
static_assert(kT2C == 128 && kOB == 128, "the wave layout assumes a 128 x 128 block");
static_assert(2 * kT2Lds <= 160 * 1024, "two workgroups per CU (gfx950 LDS)");
constexpr int kLinvFloats = kOB * kOB;

// Two-level L11^-1 of the block's 128 x 128 unit-lower factor (r05), row-major 128 x 128 into Linv[b]:
// the four 32 x 32 diagonal blocks inverted (Linv_jj), the blocks below them as L_ij, zeros above.
// lu_trail128_kernel's prologue then forms U12 block row by block row, U_j = Linv_jj (A_j - sum_{i<j}
// L_ji U_i): substitution between the 32-row blocks, explicit inverses only within them.  (r04: the
// explicit inverse of the whole 128 x 128 factor; its residual grows with kappa(L11) where
// substitution's does not -- the factorization's backward error was 1.6-1.8x MKL sgetrf's on the
// KKT matrices, 0.95-1.0x with the two-level form: tools/lu_accuracy_sim.py,
// profiles/r05_lu_accuracy_sim_N2000.txt.)  Thread j computes column j % 32 of its diagonal block by
// forward substitution (one fmaf chain per entry, L broadcast from LDS) and writes column j.
// perm != nullptr (r04, look-ahead): a third wave builds the block's composed permutation (what
// lu_block_perm_kernel does) beside the substitution, one launch less on the critical path.
constexpr int kLd = 32;  // diagonal block of the two-level inverse
__global__ __launch_bounds__(kOB + 64) void lu_linv_kernel(int N, int P, const float* A, float* Linv, const int* piv,
                                                         int* perm, int cend) {
  __shared__ __attribute__((aligned(16))) float L[kOB][kOB + 4];
  __shared__ int pvs[kPermMax], prow[2 * kPermMax], pcur[2 * kPermMax], pcnt[1];
  const int j = threadIdx.x;
  const size_t b = blockIdx.x;
  const float* Ab = A + b * (size_t)N * N;
  if (j >= kOB) {  // the permutation wave
    const int nbk = cend - P, lane = j - kOB;
    if (perm)
      for (int i = lane; i < nbk; i += 64) pvs[i] = piv[b * N + P + i] - 1;
    __syncthreads();  // (the block's one barrier: L staged)
    if (!perm) return;
    build_row_perm(pvs, P, nbk, prow, pcur, pcnt, kOB / 64, false);
    int* out = perm + b * kPermInts;
    for (int i = lane; i < 2 * kPermMax; i += 64) { out[i] = prow[i]; out[2 * kPermMax + i] = pcur[i]; }
    if (lane == 0) out[4 * kPermMax] = *pcnt;
    return;
  }
  // the 128 x 128 block in four batches of 32 row loads per thread (a batch's loads all in flight
  // together; r03 first form: a 128-iteration load -> LDS-store loop, one latency after another)
  constexpr int kLB = 32;
#pragma unroll
  for (int h0 = 0; h0 < kOB * kOB; h0 += kLB * kOB) {
    float v[kLB];
#pragma unroll
    for (int i = 0; i < kLB; ++i) {
      const int idx = h0 + i * kOB + j, r = idx / kOB, c = idx % kOB;
      v[i] = Ab[(size_t)(P + r) * N + P + c];
    }
#pragma unroll
    for (int i = 0; i < kLB; ++i) {
      const int idx = h0 + i * kOB + j, r = idx / kOB, c = idx % kOB;
      L[r][c] = c < r ? v[i] : 0.f;
    }
  }
  __syncthreads();
  const int d0 = j & ~(kLd - 1), jj = j - d0;  // this column's diagonal block [d0, d0 + 32)
  float x[kLd];
#pragma unroll
  for (int i = 0; i < kLd; ++i) {
    float s = i == jj ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < i; ++k) s = fmaf(-L[d0 + i][d0 + k], x[k], s);
    x[i] = i < jj ? 0.f : s;
  }
  float* out = Linv + b * (size_t)kLinvFloats;
#pragma unroll
  for (int bi = 0; bi < kOB / kLd; ++bi)
#pragma unroll
    for (int t = 0; t < kLd; ++t) {
      const int i = bi * kLd + t;
      out[i * kOB + j] = kLd * bi == d0 ? x[t] : (kLd * bi > d0 ? L[i][j] : 0.f);
    }
}

// Fused row interchanges, U12 = L11^-1 A12 and A22 -= L21 U12 (rank 128) for the columns right of
// [P, P + 128).  One workgroup per (instance, 128-column strip), all trailing rows; 4 waves and 72 KB
// of LDS, so TWO workgroups share a CU (r04; the r03 form ran one 8-wave workgroup per CU, whose
// waves all reached their output phase together behind one barrier while the MFMA pipe idled:
// tools/lubench128.hip, profiles/r04_lubench128_paired.txt).  The block's 128 interchanges
// (composed by lu_block_perm_kernel: block row P + i takes row pcur[i], each displaced row below the
// block takes an original block row) get no pass of their own over these columns: the loads gather
// through the permutation, and the block rows -- the only sources of displaced rows -- are
// overwritten (with U12) after the last step's loads.  A displaced row finds its source in O(1):
// sources sorted by row (dsrc), the rank of a step's first displaced row (dpre) plus the popcount
// of the step's bitmap below the row.  (perm == nullptr: no interchanges, tools/lubench128.hip.)
//   prologue: U12 = L11^-1 A12 on MFMA by 32-row blocks (two-level, r05: U_j = Linv_jj (A_j -
//             sum_{i<j} L_ji U_i); wave w: strip columns [32w, 32w + 32), no exchange between waves),
//             transposed into LDS, then each wave's MFMA operand for the main loop -- column 32w + il,
//             k in [64h, 64h + 64): 64 registers -- kept in registers for the whole loop;
//   main loop: 32-row steps; wave w owns columns [32w, 32w + 32) of a step (v_mfma_f32_32x32x2f32,
//             64 per step, the first on an inline-zero C, L21 fragments read two k-groups ahead,
//             U12 from registers).  L21 and the product tile are double-buffered in LDS, so a step
//             needs ONE barrier: per wave, step t = issue the loads of A22 (t + 1) and L21 (t + 2); the
//             MFMAs; product -> Cb[t & 1]; L21 (t + 1) -> Ls[(t + 1) & 1]; barrier; out = A22 -
//             product for step t (row-contiguous global stores, the A22 values already in the
//             registers of the storing thread).
// Main loop: the same MFMA chains, products and subtractions as the r03 kernel.
// Strips of one instance are consecutive logical ids on one XCD (its L2 serves the L21 re-reads).
// DIAG (tools/lubench128.hip only): 1 = no MFMAs in the main loop, 2 = no global A22 / L21 traffic in it.
template <bool VEC, int DIAG = 0>
__global__ __launch_bounds__(kT2Threads, 2) void lu_trail128_kernel(int N, int P, int ntc, int tc0, float* A,
                                                                    const float* Linv, const int* perm) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ls0 = sm;                      // 2 x [kT2S rows][kT2K]: L21 of a step
  float* Cb0 = sm + 2 * kT2S * kT2K;    // 2 x [kT2S rows][kT2CS]: product of a step
  float* Ut = sm;                       // after the prologue: U12^T [128 cols][kT2K]
  int* bsrc = reinterpret_cast<int*>(sm + kT2AreaFloats);  // [128] source row of block row P + i
  int* tdst = bsrc + kPermMax;          // [128] displaced rows and
  int* tsrc = tdst + kPermMax;          // [128] their sources, as given;
  int* dsrc = tsrc + kPermMax;          // [128] the sources sorted by displaced row
  unsigned* dbits = reinterpret_cast<unsigned*>(dsrc + kPermMax);  // 1 word per step: displaced rows
  unsigned char* dpre = reinterpret_cast<unsigned char*>(dbits + kT2BitWords);  // rank of a step's first
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const size_t b = (size_t)(logical / ntc);
  const int tc = tc0 + logical % ntc;  // (this launch's strips: [tc0, tc0 + ntc))
  float* Ab = A + b * (size_t)N * N;
  const int c0 = P + kOB, cb = c0 + tc * kT2C;
  const int nsteps = (N - c0 + kT2S - 1) / kT2S;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NT = kT2Threads;

  typedef typename std::conditional<VEC, float4, float>::type VT;
  constexpr int W = VEC ? 4 : 1;
  constexpr int kCQ = kT2S * kT2C / W / NT;   // A22 accesses per thread per step
  constexpr int kLQ = kT2S * kOB / W / NT;    // L21 accesses per thread per step
  constexpr int CPR = kT2C / W, LPR = kOB / W;
  // main-loop loads: unconditional, from a clamped (valid) address.  Rows >= N / columns >= N only
  // feed products that are never stored, so they need no zero fill -- and a load with no select
  // stays out of a branch, which keeps the compiler's vmcnt waits exact (a conditional load costs a
  // full vmcnt(0) drain at every later use).
  auto ldu = [&](int row, int col) -> VT {
    const float* p = Ab + (size_t)row * N + col;
    if constexpr (VEC) return *reinterpret_cast<const float4*>(p);
    else return *p;
  };

  // ---- the permutation (displaced rows are >= c0 and distinct; <= 128 of them)
  const int ndisp = perm ? perm[b * kPermInts + 4 * kPermMax] - kOB : 0;
  {
    const int* pb = perm + b * kPermInts;
    if (tid < kOB) bsrc[tid] = perm ? pb[2 * kPermMax + tid] : P + tid;
    if (tid < ndisp) { tdst[tid] = pb[kOB + tid]; tsrc[tid] = pb[2 * kPermMax + kOB + tid]; }
    if (perm)  // (the tables are sized for N <= kLuMaxN: the interchange-free form never reads them)
      for (int w = tid; w < nsteps + 2; w += NT) { dbits[w] = 0u; dpre[w] = 0; }  // (+ one past the end)
  }
  __syncthreads();
  int drank = 0, dd = 0;
  if (tid < ndisp) {
    dd = tdst[tid] - c0;
    for (int j = 0; j < ndisp; ++j) drank += tdst[j] - c0 < dd;
    dsrc[drank] = tsrc[tid];
    atomicOr(&dbits[dd >> 5], 1u << (dd & 31));
  }
  __syncthreads();
  if (tid < ndisp && __builtin_popcount(dbits[dd >> 5] & ((1u << (dd & 31)) - 1u)) == 0)
    dpre[dd >> 5] = (unsigned char)drank;
  // (published by the prologue's barriers)

  // ---- prologue (r05, two-level): U12 = L11^-1 A12 on this strip by 32-row blocks,
  // U_j = Linv_jj (A_j - sum_{i<j} L_ji U_i) (lu_linv_kernel's layout: Linv_jj on the diagonal, L_ji
  // below), carried negated -- acc = -A_j + sum L_ji U_i, U_j = -(Linv_jj acc), exact sign flips, so
  // no operand needs negating (and lu_trail256_kernel can stage L rows straight from A by LDS-DMA).  Wave w owns the strip's columns [32w, 32w + 32) for all 128 rows, so it needs no other
  // wave's result: its U_i are accumulator tiles (lane half h: rows 8q + 4h + r of the block, column
  // il), and the MFMA k index runs over exactly those rows -- U_i is the B operand straight from
  // registers, the matching L entries (four consecutive k) one 16-B LDS read.  A_j is the first
  // MFMA's C operand (the gathered block rows, loaded in accumulator layout).
  const float* Lb = Linv + b * (size_t)kLinvFloats;
  float* Lt = sm;  // [128 rows][kT2LK]: Lb staged
  {
    float4 lv[kOB * kOB / 4 / NT];
#pragma unroll
    for (int q = 0; q < kOB * kOB / 4 / NT; ++q) {
      const int e = tid + NT * q;
      lv[q] = *reinterpret_cast<const float4*>(Lb + (size_t)(e / (kOB / 4)) * kOB + (e % (kOB / 4)) * 4);
    }
#pragma unroll
    for (int q = 0; q < kOB * kOB / 4 / NT; ++q) {
      const int e = tid + NT * q;
      *reinterpret_cast<float4*>(Lt + (e / (kOB / 4)) * kT2LK + (e % (kOB / 4)) * 4) = lv[q];
    }
  }
  floatx16 u[4];
  {
    // (columns >= N: clamped loads, never stored -- a column of U12 feeds only its own column)
    const int colc = min(cb + 32 * wave + il, N - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        u[j][v] = Ab[(size_t)bsrc[32 * j + 8 * (v >> 2) + 4 * h + (v & 3)] * N + colc];
  }
  __syncthreads();  // Lt staged
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    floatx16 acc = -u[j];
#pragma unroll
    for (int i = 0; i < j; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 l4 = *reinterpret_cast<const float4*>(Lt + (32 * j + il) * kT2LK + 32 * i + 8 * q + 4 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(l4, r), u[i][4 * q + r], acc, 0, 0, 0);
      }
    const floatx16 zero = {};
    floatx16 o = zero;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 l4 = *reinterpret_cast<const float4*>(Lt + (32 * j + il) * kT2LK + 32 * j + 8 * q + 4 * h);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(l4, r), acc[4 * q + r], (q == 0 && r == 0) ? zero : o, 0, 0, 0);
    }
    u[j] = -o;
  }
  __syncthreads();  // the pass tiles consumed: U12^T over them
  // accumulator v of tile j <-> U12 row 32j + 8(v/4) + 4h + v%4, strip column 32w + il
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) Ut[(wave * 32 + il) * kT2K + 32 * j + 8 * (v >> 2) + 4 * h + (v & 3)] = u[j][v];
  __syncthreads();
  const int wc = wave * 32;
  float4 ub[kOB / 8];  // U12[64h + 4sg + 0..3][wc + il]: this wave's MFMA operand for every step
#pragma unroll
  for (int sg = 0; sg < kOB / 8; ++sg)
    ub[sg] = *reinterpret_cast<const float4*>(Ut + (wc + il) * kT2K + (kOB / 2) * h + 4 * sg);
  __syncthreads();  // Ut consumed: Ls / Cb from here on

  // ---- main loop
  auto loadC = [&](int step, VT (&c)[kCQ]) {
    const unsigned m = perm ? __builtin_amdgcn_readfirstlane(dbits[step]) : 0u;
    const int pre = perm ? __builtin_amdgcn_readfirstlane((int)dpre[step]) : 0;
    int srow[kCQ];
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {  // (every lane reads a table entry: no branch around the loads)
      const int ro = (tid + NT * q) / CPR;
      srow[q] = dsrc[(pre + __builtin_popcount(m & ((1u << ro) - 1u))) & (kPermMax - 1)];
    }
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, ro = e / CPR, row = c0 + step * kT2S + ro, col = cb + (e % CPR) * W;
      const int src = ((m >> ro) & 1u) ? srow[q] : row;
      c[q] = ldu(min(src, N - 1), min(col, N - W));
    }
  };
  auto loadL = [&](int step, VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q, row = c0 + step * kT2S + e / LPR;
      l[q] = ldu(min(row, N - 1), P + (e % LPR) * W);
    }
  };
  auto writeL = [&](float* Ls, const VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q;
      if constexpr (VEC) *reinterpret_cast<float4*>(Ls + (e / LPR) * kT2K + (e % LPR) * W) = l[q];
      else Ls[(e / LPR) * kT2K + (e % LPR)] = l[q];
    }
  };
  // (the result overwrites c in place and is stored from there: a store's data registers stay busy
  // until the store completes, and c is not reloaded until the next step but one)
  auto storeOut = [&](int step, const float* Cb, VT (&c)[kCQ]) {
    VT pr[kCQ];  // every product read before the first subtract: one LDS latency, not kCQ
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q;
      const float* src = Cb + (e / CPR) * kT2CS + (e % CPR) * W;
      if constexpr (VEC) pr[q] = *reinterpret_cast<const float4*>(src);
      else pr[q] = *src;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, row = c0 + step * kT2S + e / CPR, col = cb + (e % CPR) * W;
      if constexpr (VEC) {
        c[q].x -= pr[q].x; c[q].y -= pr[q].y; c[q].z -= pr[q].z; c[q].w -= pr[q].w;
      } else {
        c[q] -= pr[q];
      }
      if (row < N && col < N) {
        if constexpr (VEC) *reinterpret_cast<float4*>(Ab + (size_t)row * N + col) = c[q];
        else Ab[(size_t)row * N + col] = c[q];
      }
    }
  };
  auto chain = [&](const float* Ls) -> floatx16 {
    floatx16 acc = {};
    if constexpr (DIAG != 1) {
      // L21 fragments read two k-groups ahead of their MFMAs (pinned: the scheduler otherwise waits
      // for each read right before its four MFMAs)
      const floatx16 zero = {};  // the first MFMA takes an inline-zero C operand (no zeroing moves)
      const float* lrow = Ls + il * kT2K + (kOB / 2) * h;
      float4 fa[kOB / 8];
      __builtin_amdgcn_sched_barrier(0);
      fa[0] = *reinterpret_cast<const float4*>(lrow);
      fa[1] = *reinterpret_cast<const float4*>(lrow + 4);
#pragma unroll
      for (int sg = 0; sg < kOB / 8; ++sg) {
        if (sg + 2 < kOB / 8) fa[sg + 2] = *reinterpret_cast<const float4*>(lrow + 4 * (sg + 2));
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa[sg], s4), get4(ub[sg], s4), (sg == 0 && s4 == 0) ? zero : acc,
                                                     0, 0, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int sg = 0; sg < kOB / 8 - 2; ++sg) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  };

  // step t (cc = A22 (t), loaded during step t - 1; lw = L21 (t + 1), loaded during step t - 1)
  auto body = [&](int step, VT (&cc)[kCQ], VT (&cn)[kCQ], const VT (&lw)[kLQ], VT (&lnext)[kLQ]) {
    const float* Ls = Ls0 + (step & 1) * (kT2S * kT2K);
    float* Cb = Cb0 + (step & 1) * (kT2S * kT2CS);
    if (DIAG != 2) {  // (past the last step: clamped rows, never used)
      loadC(step + 1, cn);
      loadL(step + 2, lnext);
    }
    const floatx16 acc = chain(Ls);
#pragma unroll
    for (int v = 0; v < 16; ++v) Cb[(8 * (v >> 2) + 4 * h + (v & 3)) * kT2CS + wc + il] = acc[v];
    writeL(Ls0 + ((step + 1) & 1) * (kT2S * kT2K), lw);
    __syncthreads();  // Cb[t & 1] = product (t), Ls[(t + 1) & 1] = L21 (t + 1); Ls[t & 1] consumed
    if (DIAG != 2) storeOut(step, Cb, cc);
  };

  if constexpr (VEC) {
    VT c0r[kCQ], c1r[kCQ], la[kLQ], lb[kLQ];
    loadC(0, c0r);
    loadL(0, la);
    loadL(1, lb);
    writeL(Ls0, la);
    __syncthreads();
    // pairs of steps, the odd last one after the loop: no conditional body inside the loop, whose
    // merge would make the compiler copy the register sets (waiting on their loads to do so)
    int step = 0;
    for (; step + 1 < nsteps; step += 2) {
      body(step, c0r, c1r, lb, la);
      body(step + 1, c1r, c0r, la, lb);
    }
    if (step < nsteps) body(step, c0r, c1r, lb, la);
  } else {
    // scalar path (N % 4 != 0: 16 single-float accesses per thread and array): one register set
    // each, the next step's loads issued after the output (the double sets spill here)
    VT c[kCQ], l[kLQ];
    loadC(0, c);
    loadL(0, l);
    writeL(Ls0, l);
    loadL(1, l);
    __syncthreads();
    for (int step = 0; step < nsteps; ++step) {
      float* Cb = Cb0 + (step & 1) * (kT2S * kT2CS);
      const floatx16 acc = chain(Ls0 + (step & 1) * (kT2S * kT2K));
#pragma unroll
      for (int v = 0; v < 16; ++v) Cb[(8 * (v >> 2) + 4 * h + (v & 3)) * kT2CS + wc + il] = acc[v];
      writeL(Ls0 + ((step + 1) & 1) * (kT2S * kT2K), l);
      __syncthreads();
      if (DIAG != 2) {
        storeOut(step, Cb, c);
        loadC(step + 1, c);
        loadL(step + 2, l);
      }
    }
  }
  __syncthreads();  // every gathered load of a block row has completed: U12 to the block rows
  if (cb + wc + il < N) {
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg) {
      const int i = (kOB / 2) * h + 4 * sg;
      float* dst = Ab + (size_t)(P + i) * N + cb + wc + il;
      dst[0] = ub[sg].x;
      dst[(size_t)N] = ub[sg].y;
      dst[2 * (size_t)N] = ub[sg].z;
      dst[3 * (size_t)N] = ub[sg].w;
    }
  }
}

// ---- Paired blocks (r05): one rank-256 update of the far columns per two 128-column blocks ----
// At rank 128 the trailing update streams A22 at 32 flop/B: 157 TF/s of fp32 MFMA would need ~9.8 TB/s
// of HBM for A22 alone, so lu_trail128_kernel is memory-bound (~0.6 of MFMA).  With the left
// interchanges deferred (N <= 2048), blocks t (even) and t + 1 are factored back to back -- block t
// updating only block t + 1's columns (lu_trail128_kernel, strip 0) -- and everything right of block
// t + 1 then gets ONE update with both blocks' factors:
//   U12 = L^-1 A12 over the pair's 256 rows (two-level: 32-row blocks, Linv_jj from each block's
//         lu_linv_kernel buffer; L = [[L11_t, 0], [L_{t+1,t}, L11_{t+1}]], L_{t+1,t} = block t's
//         multipliers in block t + 1's rows);
//   A22 -= [L21_t  L21_{t+1}] U12   (rank 256: 64 flop/B, MFMA-bound).
// Interchanges: the far columns have had neither block's applied -- A22 and A12 rows gather through the
// pair's composed permutation (both blocks' own permutations composed); block t's columns
// have had block t + 1's interchanges deferred too, so L21_t rows gather through block t + 1's own
// permutation.  A displaced row's source is always one of the pair's 256 block rows, which take U12
// only after the last step's loads (as in lu_trail128_kernel).
constexpr int kR2 = 2 * kOB;                 // rank of the paired update
constexpr int kP2K = kR2 + 4;                // LDS stride (k) of its L21 tiles and staged L rows
constexpr int kD2Threads = 256;              // lu_trail256_kernel: 4 waves, two workgroups per CU,
constexpr int kD2S = 32;                     //   rows per step,
constexpr int kD2Rows = 2048 + 2 * kD2S;     //   row-source table (N <= 2048, whole steps + one)
constexpr int kP2BitWords = (2048 + 31) / 32 + 4;  // one per step (pairing only with the deferred left pass)
constexpr int kP2AreaFloats = 2 * kD2S * kP2K;     // the L21 ring (two steps) = the prologue's 64 staged L rows
constexpr size_t kP2Lds = (size_t)kP2AreaFloats * sizeof(float) +
                          (size_t)(kR2 + kD2Rows + 3 * kPermMax + kP2BitWords) * sizeof(int) +
                          (size_t)((kP2BitWords + 3) & ~3);
static_assert(2 * kP2Lds <= 160 * 1024, "two workgroups per CU (gfx950 LDS)");

// The paired far update: per (instance, 128-column strip right of the pair), all rows below it.  r05
// third form: TWO workgroups of four waves per CU (2 waves per SIMD), 32-row steps, wave w owning the
// strip's columns [32w, 32w + 32).  (The first form, four waves with the product tile through LDS, and
// the second, one 8-wave workgroup per CU with 64-row steps, ran at ~0.6 of MFMA: their prologue was
// computed twice (both row halves) and a step's memory work and barrier stalled the whole CU --
// profiles/r05_lubench256.txt.)
//   prologue: U12 = L^-1 A12 over the pair's 256 rows, two-level, carried negated (see
//             lu_trail128_kernel's prologue), 64 staged L rows (two 32-row blocks) at a time; wave w
//             computes only its own 32 columns.  U12 stays in registers in accumulator layout (block
//             j, register v: row 32j + 8(v/4) + 4h + v%4, column il) and is the main loop's B operand
//             as it is: the k index of an MFMA pair is (32j + 8q + r, 32j + 8q + 4 + r), lane half h
//             taking the second, so the matching L21 entries (four consecutive k) are one 16-B LDS read;
//   main loop: the step's A22 tile is the first MFMA's C operand, loaded straight into accumulator
//             layout (one dword per lane, two 128-B row pieces per instruction), and the result is
//             stored from the accumulators (buffer stores; rows / columns >= N dropped by the range
//             check).  L21 comes by LDS-DMA into a two-step ring (one barrier per step).  The memory
//             work of step s + 1 (A22 loads, L21 DMA) and the stores of step s - 1 ride inside step s's
//             128-MFMA chain; three accumulator-register sets rotate (A22 (s) / result (s - 1) being
//             stored / A22 (s + 1) being loaded): the compiler holds a store's data registers until
//             the store completes (gfx9: one vmcnt for loads and stores).  The L21 fragments are read
//             by inline-asm ds_read_b128 with explicit lgkmcnt waits: the compiler treats every LDS
//             read as possibly aliasing an in-flight LDS-DMA and would drain vmcnt before it (the ring
//             slot read is never the one the DMA fills).
// Interchanges: A22 and A12 rows gather through the pair's composed permutation -- a row-source table
// over [P, N) composed in LDS at the start from the two blocks' own permutations (perm0, perm1: one
// scatter each, no replay of the 256 pivots); L21's block-t half gathers through block t + 1's own
// permutation.  A displaced row's source is one of the pair's 256 rows, which take U12 only after the
// last step's loads.
// Linv0 / Linv1: the two blocks' lu_linv_kernel buffers.  N % 4 == 0, 16-B aligned rows, N <= 2048
// (the host checks).  MODE: tools/lubench256.hip's timing diagnostics only (results meaningless):
// 4 = no main-loop memory work, 8 = one VALU op per main-loop MFMA instead, 16 = no prologue MFMAs.
template <int MODE = 0>
__global__ __launch_bounds__(kD2Threads, 2) void lu_trail256_kernel(int N, int P, int ntc, int tc0, float* A,
                                                                    const float* Linv0, const float* Linv1,
                                                                    const int* perm0, const int* perm1) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ls0 = sm;                       // 2 x [32 rows][kP2K]: L21 of a step
  float* Lt = sm;                        // prologue: 64 staged L rows [64][kP2K]
  int* bsrc = reinterpret_cast<int*>(sm + kP2AreaFloats);  // [256] source row of pair row P + i, then
  int* rowsrc = bsrc + kR2;              // [kD2Rows] of row c0 + i (one table: the composed permutation)
  int* tdst1 = rowsrc + kD2Rows;         // [128] block t + 1's displaced rows,
  int* tsrc1 = tdst1 + kPermMax;         // [128] their sources,
  int* dsrc1 = tsrc1 + kPermMax;         // [128] sorted
  unsigned* dbits1 = reinterpret_cast<unsigned*>(dsrc1 + kPermMax);  // one word per step
  unsigned char* dpre1 = reinterpret_cast<unsigned char*>(dbits1 + kP2BitWords);
  constexpr bool kNoMem = (MODE & 4) != 0, kNoMfma = (MODE & 8) != 0, kNoPro = (MODE & 16) != 0;
  // where the memory work rides in the 32 fragment groups of a step's chain: the A22 loads of step s + 1
  // in groups 2-5, its L21 DMA in 6-9, the stores of step s - 1 in 14, 17, 20, 23 (profiles/
  // r05_lubench256_sched.txt: 1-4 / 5-8 / 9-12 was 1-4 % slower, other spreads within 1 %)
  constexpr int kC0 = 2, kL0 = 6, kS0 = 14, kSs = 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const size_t b = (size_t)__builtin_amdgcn_readfirstlane(logical / ntc);  // (uniform: scalar rsrc)
  const int tc = __builtin_amdgcn_readfirstlane(tc0 + logical % ntc);
  float* Ab = A + b * (size_t)N * N;
  const int P1 = P + kOB, c0 = P + kR2, cb = c0 + tc * kT2C;
  const int nsteps = (N - c0 + kD2S - 1) / kD2S;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NT = kD2Threads, NW = NT / 64;
  // the instance's matrix as a buffer: rows >= N land past its end (loads 0, stores dropped).  (Made
  // where it is used: a descriptor captured by reference stayed in private memory, and every buffer
  // operation became a waterfall loop over a "divergent" descriptor.)
  float* Abu;  // Ab, provably wave-uniform (a pointer derived from it was treated as divergent)
  {
    const uint64_t ab = reinterpret_cast<uint64_t>(Ab);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)ab), hi = __builtin_amdgcn_readfirstlane((unsigned)(ab >> 32));
    Abu = reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
  }
#define IADMM_RS __builtin_amdgcn_make_buffer_rsrc(Abu, 0, N * N * 4, 0x00020000)
  const unsigned kOut = 0x7ffffff0u;     // an offset past the end: the store is dropped

  // ---- the pair's row map, bsrc[x - P] (x in [P, c0 + kD2S (nsteps + 1))): the row whose content row x
  // holds after both blocks' interchanges -- identity, then block t's (rowid -> cur), then block t + 1's
  // on top (its sources read through the map before any of its writes); rows >= N clamped (the last
  // step's look-ahead loads read one step past the end).  lu_block_perm layout: rowid [0, cnt), cur
  // [256, 256 + cnt), cnt at 512.
  const int* pa = perm0 + b * kPermInts;
  const int* qb = perm1 + b * kPermInts;
  const int cnta = pa[4 * kPermMax], ndisp1 = qb[4 * kPermMax] - kOB;
  for (int x = tid; x < kR2 + kD2S * (nsteps + 1); x += NT) bsrc[x] = min(P + x, N - 1);
  if (tid < ndisp1) { tdst1[tid] = qb[kOB + tid]; tsrc1[tid] = qb[2 * kPermMax + kOB + tid]; }
  for (int w = tid; w < nsteps + 2; w += NT) { dbits1[w] = 0u; dpre1[w] = 0; }
  __syncthreads();
  for (int i = tid; i < cnta; i += NT) bsrc[pa[i] - P] = pa[2 * kPermMax + i];
  __syncthreads();
  const int cntb = ndisp1 + kOB;  // (<= 256 = NT)
  const int vb1 = tid < cntb ? bsrc[qb[2 * kPermMax + tid] - P] : 0;
  __syncthreads();
  if (tid < cntb) bsrc[qb[tid] - P] = vb1;
  int drank1 = 0, dd1 = 0;
  if (tid < ndisp1) {
    dd1 = tdst1[tid] - c0;
    for (int j = 0; j < ndisp1; ++j) drank1 += tdst1[j] - c0 < dd1;
    dsrc1[drank1] = tsrc1[tid];
    atomicOr(&dbits1[dd1 >> 5], 1u << (dd1 & 31));
  }
  __syncthreads();
  if (tid < ndisp1 && __builtin_popcount(dbits1[dd1 >> 5] & ((1u << (dd1 & 31)) - 1u)) == 0)
    dpre1[dd1 >> 5] = (unsigned char)drank1;
  // (published by the prologue's barriers)

  // ---- prologue: U_j = Linv_jj (A_j - sum_{i<j} L_ji U_i), j = 0..7, carried negated; this wave's columns
  floatx16 u[8];
  const int col = cb + 32 * wave + il;
  const int colc = min(col, N - 1);  // (columns >= N: clamped, never stored)
  auto mfma = [](float a, float b_, const floatx16& c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b_, c, 0, 0, 0); };
  auto solve_row_block = [&](int j) {  // staged L rows: block j's are Lt rows 32 (j & 1) + [0, 32)
    const float* lr = Lt + (32 * (j & 1) + il) * kP2K + 4 * h;
    floatx16 acc = -u[j];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i >= j) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 l4 = *reinterpret_cast<const float4*>(lr + 32 * i + 8 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma(get4(l4, r), u[i][4 * q + r], acc);
      }
    }
    const floatx16 zero = {};
    floatx16 o = zero;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 l4 = *reinterpret_cast<const float4*>(lr + 32 * j + 8 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) o = mfma(get4(l4, r), acc[4 * q + r], (q == 0 && r == 0) ? zero : o);
    }
    u[j] = -o;
  };
  // a staged L row (LDS-DMA, 16 B per lane): lanes 0..31 its columns [0, 128), lanes 32..63 [128, 256)
  auto stage_row = [&](int r, const float* lo_src, const float* hi_src) {
    const float* src = lane < 32 ? lo_src + 4 * lane : hi_src + 4 * (lane - 32);
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(Lt + r * kP2K), 16, 0, 0);
  };
  // every gathered A12 row of the prologue in flight at once (one memory latency, not four)
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) u[j][v] = Ab[(size_t)bsrc[32 * j + 8 * (v >> 2) + 4 * h + (v & 3)] * N + colc];
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    // pair rows [64 ph, 64 ph + 64): block t's rows hold Linv0 (columns [0, 128); the high half-row a
    // harmless copy); block t + 1's rows hold L21_t of those rows (gathered through block t + 1's
    // permutation) in [0, 128) and Linv1 in [128, 256)
    for (int r = wave; r < 2 * kD2S; r += NW) {
      const int pr = 64 * ph + r;
      if (ph < 2) {
        const float* Lb = Linv0 + b * (size_t)kLinvFloats + (size_t)pr * kOB;
        stage_row(r, Lb, Lb);
      } else {
        stage_row(r, Ab + (size_t)qb[2 * kPermMax + pr - kOB] * N + P, Linv1 + b * (size_t)kLinvFloats + (size_t)(pr - kOB) * kOB);
      }
    }
    vm_wait<0>();
    __syncthreads();
    if (!kNoPro) {
      solve_row_block(2 * ph);
      solve_row_block(2 * ph + 1);
    }
    __syncthreads();  // Lt consumed
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) u[j] = -u[j];  // -U12: acc = A22 + L21 (-U12)

  // ---- main loop
  const unsigned N4 = 4u * (unsigned)N;
  // (the lane's half-row offset 4h is laundered so that what depends on it is formed per use, not held
  // in registers across the loop; row offsets 8q + r ride in the scalar offset of each buffer access)
  // Stores past row N on a partial last step (N = 2000: rows 2000..2015 of the last 32-row step) are
  // dropped by the descriptor's range check only because gfx950 counts the SGPR soffset in it
  // (voffset + soffset >= num_records drops the access): measured on the box by
  // tools/buffer_soffset_probe.hip, profiles/r04_buffer_soffset_probe.txt ("soffset IS part of the
  // range check").  A target that excluded soffset would write the next instance's leading rows here;
  // tests/test_abi_concurrency_gpu.py::test_lu_bench_shape_repeat_bitwise (N = 2000, every instance's
  // factors and pivots) and the Stage-II envelope tests would catch that.
  auto storeQ = [&](int s, const floatx16& c, int q) {  // 4 of a step's 16 stores (s < 0: dropped)
    int h4 = 4 * h;
    asm volatile("" : "+v"(h4));
    const unsigned vb = (s >= 0 && col < N) ? (unsigned)((c0 + kD2S * s + h4) * N + col) * 4u : kOut;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      // (__float_as_uint on a copy: hipcc 7.2 lowers __builtin_bit_cast of an ext-vector element
      // reached through a reference to element 0 for every v -- all 16 stores wrote c[0])
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(float(c[4 * q + r])), IADMM_RS, vb, (int)((8 * q + r) * N4), 0);
  };
  // 2 of this wave's 8 L21 rows of step s (rows wave + 4i): the block-t half gathers through block t + 1's
  // permutation (wave-uniform: scalar table lookups), the block-(t+1) half is in place
  auto issueLQ = [&](int s, int q) {
    float* Ls = Ls0 + (s & 1) * (kD2S * kP2K);
    const bool lo = lane < 32;
    const unsigned m = __builtin_amdgcn_readfirstlane(dbits1[s]);
    const int pre = __builtin_amdgcn_readfirstlane((int)dpre1[s]);
#pragma unroll
    for (int i = 2 * q; i < 2 * q + 2; ++i) {
      const int ro = wave + NW * i, row = c0 + kD2S * s + ro;
      const int s1 = __builtin_amdgcn_readfirstlane(dsrc1[(pre + __builtin_popcount(m & ((1u << ro) - 1u))) & (kPermMax - 1)]);
      const int src = min(((m >> ro) & 1u) ? s1 : row, N - 1), rowc = min(row, N - 1);
      const unsigned voff = lo ? (unsigned)((src * N + P + 4 * lane) * 4) : (unsigned)((rowc * N + P1 + 4 * (lane - 32)) * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(IADMM_RS, (lds_void*)(Ls + ro * kP2K), 16, voff, 0, 0, 0);
    }
  };
  // 4 of a step's 16 A22 loads, gathered (one row-table read per row, no search)
  auto issueCQ = [&](int s, floatx16& c, int q) {
    int h4 = 4 * h;
    asm volatile("" : "+v"(h4));
    const int* rt = rowsrc + kD2S * s + h4;
    const unsigned cc4 = 4u * (unsigned)colc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned src = (unsigned)rt[8 * q + r];
      c[4 * q + r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(IADMM_RS, __umul24(src, N4) + cc4, 0, 0));
    }
  };
  // step s -- cc: A22 (s) in, result (s) out; co: result (s - 1), stored; cn: A22 (s + 1), loaded
  auto body = [&](int s, floatx16& cc, const floatx16& co, floatx16& cn) {
    vm_wait<0>();
    __syncthreads();  // L21 (s) everywhere; every wave past chain (s - 1): ring slot (s + 1) & 1 free
    const float* lrow = Ls0 + (s & 1) * (kD2S * kP2K) + il * kP2K + 4 * h;
    const unsigned la = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)lrow;
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v fa[kR2 / 8];  // fragment g = 4j + q: L21[row il][32j + 8q + 4h + 0..3], at byte offset 32 g
    floatx16 acc = cc;
    asm volatile("ds_read_b128 %0, %1" : "=v"(fa[0]) : "v"(la));
    asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(fa[1]) : "v"(la));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < kR2 / 8; ++g) {
      if (g + 2 < kR2 / 8) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[g + 2]) : "v"(la), "i"(32 * (g + 2)));
      // fa[g] landed (LDS operations complete in order; the other work of a group waits for its own)
      if (g + 2 < kR2 / 8) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(fa[g]));
      else if (g + 1 < kR2 / 8) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(fa[g]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[g]));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!kNoMfma) acc = mfma(fa[g][r], u[g >> 2][4 * (g & 3) + r], acc);
        else acc[r] = fmaf(fa[g][r], u[g >> 2][4 * (g & 3) + r], acc[r]);  // (hipcc 7.2 crashes on an empty chain)
      }
      if (!kNoMem && g >= kC0 && g < kC0 + 4) issueCQ(s + 1, cn, g - kC0);
      if (!kNoMem && g >= kL0 && g < kL0 + 4) issueLQ(s + 1, g - kL0);
      if (!kNoMem && g >= kS0 && g < kS0 + 4 * kSs && (g - kS0) % kSs == 0) storeQ(s - 1, co, (g - kS0) / kSs);
      __builtin_amdgcn_sched_barrier(0);
    }
    cc = acc;
  };
  floatx16 cA, cB, cX = {};  // (cX: the first step's "previous result", its stores dropped)
#pragma unroll
  for (int q = 0; q < 4; ++q) issueLQ(0, q);
#pragma unroll
  for (int q = 0; q < 4; ++q) issueCQ(0, cA, q);
  int s = 0;
  for (; s + 2 < nsteps; s += 3) {
    body(s, cA, cX, cB);
    body(s + 1, cB, cA, cX);
    body(s + 2, cX, cB, cA);
  }
  // the last one or two steps, then the last result's stores
  if (s + 1 < nsteps) {
    body(s, cA, cX, cB);
    body(s + 1, cB, cA, cX);
    if (!kNoMem)
#pragma unroll
      for (int q = 0; q < 4; ++q) storeQ(s + 1, cB, q);
  } else if (s < nsteps) {
    body(s, cA, cX, cB);
    if (!kNoMem)
#pragma unroll
      for (int q = 0; q < 4; ++q) storeQ(s, cA, q);
  } else if (!kNoMem) {
#pragma unroll
    for (int q = 0; q < 4; ++q) storeQ(s - 1, cX, q);
  }
  vm_wait<0>();
  __syncthreads();  // every gathered load of a pair row has completed: U12 to the pair's rows
  if (col < N) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) Ab[(size_t)(P + 32 * j + 8 * (v >> 2) + 4 * h + (v & 3)) * N + col] = -u[j][v];
  }
}
#undef IADMM_RS

// Solve (P^T L U) x = b in place for one instance per workgroup.
constexpr int kDS = kSolveBlk + 1;  // LDS stride of the staged diagonal block
// VEC (N % 4 == 0, 16-B aligned factors): block bounds are multiples of 4, rows 16-B aligned.
// NT threads per workgroup: 256 (4 workgroups per CU) when the batch fills the CUs four times
// over, 512 / 1024 for smaller batches (config 4's 256-instance chunks: one workgroup per CU, so
// 16 waves instead of 4 stream its rows; the block loop spreads over any number of waves).
template <bool VEC, int NT = kSolveThreads>
__global__ __launch_bounds__(NT, NT == 256 ? 4 : (NT == 512 ? 2 : 1)) void lu_solve_kernel(int N, const float* LU, const int* piv,
                                                              float* X) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* x = sm;                  // N
  float* s = x + N;               // kSolveBlk partial sums
  float* D = s + kSolveBlk;       // kSolveBlk x kDS diagonal block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* M = LU + b * (size_t)N * N;
  float* xb = X + b * N;
#pragma unroll 8
  for (int i = tid; i < N; i += NT) x[i] = xb[i];
  __syncthreads();
  // The row interchanges (P b) are applied lazily, block by block: interchange i touches positions i
  // and piv[i] - 1 >= i only, so positions below k0 are final once those of rows < k0 are done.  Wave 0
  // applies a block's 64 (pivots loaded once per block, broadcast by shuffle) while the other waves'
  // dot products read only x[0, k0).  (r03: one thread looping over all N with a global load per
  // interchange was a serial chain of N memory latencies at the start of every solve.)
  for (int pass = 0; pass < 2; ++pass) {  // 0: forward with unit L, 1: backward with U
    const int nblk = (N + kSolveBlk - 1) / kSolveBlk;
    for (int bb = 0; bb < nblk; ++bb) {
      const int k0 = pass == 0 ? bb * kSolveBlk : max(0, N - (bb + 1) * kSolveBlk);
      const int k1 = pass == 0 ? min(N, k0 + kSolveBlk) : N - bb * kSolveBlk;
      const int nbk = k1 - k0;
      // the diagonal block: every thread issues its loads at once (clamped, valid addresses; the
      // entries past nbk are never read), the LDS writes after the dot products below
      constexpr int kDQ = kSolveBlk * kSolveBlk / NT;
      {
        float dreg[kDQ];
#pragma unroll
        for (int q = 0; q < kDQ; ++q) {
          const int idx = tid + NT * q, r = min(idx / kSolveBlk, nbk - 1), c = min(idx % kSolveBlk, nbk - 1);
          dreg[q] = M[(size_t)(k0 + r) * N + k0 + c];
        }
#pragma unroll
        for (int q = 0; q < kDQ; ++q) {
          const int idx = tid + NT * q;
          D[(idx / kSolveBlk) * kDS + idx % kSolveBlk] = dreg[q];
        }
      }
      if (pass == 0 && wave == 0) {
        const int pv = piv[b * N + k0 + min(lane, nbk - 1)] - 1;
        for (int j = 0; j < nbk; ++j) {
          const int p = __builtin_amdgcn_readlane(pv, j);
          if (lane == 0 && p != k0 + j) { const float t = x[k0 + j]; x[k0 + j] = x[p]; x[p] = t; }
        }
      }
      // prefix (forward) / suffix (backward) dot products of the block rows with x: all rows of a
      // block share the column range, so a wave takes 4 rows at a time (16-B loads, 8 in flight
      // per lane, x read once for the 4): one memory latency per 4 rows instead of per row.
      const int j0 = pass == 0 ? 0 : k1, j1 = pass == 0 ? k0 : N;
      if constexpr (VEC) {
        const float4* x4 = reinterpret_cast<const float4*>(x);
        const int q0 = j0 >> 2, q1 = j1 >> 2;
        for (int g = wave * 4; g < nbk; g += nw * 4) {
          const float4* r4[4];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            r4[rr] = reinterpret_cast<const float4*>(M + (size_t)(k0 + min(g + rr, nbk - 1)) * N);
          float d[4] = {0.f, 0.f, 0.f, 0.f};
          auto dot4 = [](const float4& u, const float4& w, float acc) {
            acc = fmaf(u.x, w.x, acc); acc = fmaf(u.y, w.y, acc);
            acc = fmaf(u.z, w.z, acc); return fmaf(u.w, w.w, acc);
          };
          int q = q0 + lane;
          for (; q + 64 < q1; q += 128) {
            const float4 b0 = x4[q], b1 = x4[q + 64];
            float4 a0[4], a1[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) { a0[rr] = r4[rr][q]; a1[rr] = r4[rr][q + 64]; }
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) d[rr] = dot4(a1[rr], b1, dot4(a0[rr], b0, d[rr]));
          }
          if (q < q1) {
            const float4 b0 = x4[q];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) d[rr] = dot4(r4[rr][q], b0, d[rr]);
          }
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const float t = wave_sum(d[rr]);
            if (lane == 0 && g + rr < nbk) s[g + rr] = t;
          }
        }
      } else {
        for (int i = wave; i < nbk; i += nw) {
          const float* row = M + (size_t)(k0 + i) * N;
          float d = 0.f;
          for (int j = j0 + lane; j < j1; j += 64) d = fmaf(row[j], x[j], d);
          d = wave_sum(d);
          if (lane == 0) s[i] = d;
        }
      }
      __syncthreads();
      if (wave == 0) {
        float v = lane < nbk ? x[k0 + lane] - s[lane] : 0.f;
        if (pass == 0) {
          for (int j = 0; j < nbk; ++j) {
            const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
            if (lane > j && lane < nbk) v = fmaf(-D[lane * kDS + j], xj, v);
          }
        } else {
          for (int j = nbk - 1; j >= 0; --j) {
            const float vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j)) / D[j * kDS + j];
            if (lane == j) v = vj;
            if (lane < j) v = fmaf(-D[lane * kDS + j], vj, v);
          }
        }
        if (lane < nbk) x[k0 + lane] = v;
      }
      __syncthreads();
    }
  }
#pragma unroll 8
  for (int i = tid; i < N; i += NT) xb[i] = x[i];
}

// info[b] = 0 before a factorization (a kernel rather than a memset node: r05)
__global__ void lu_info_zero_kernel(int64_t B, int* info) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < B) info[i] = 0;
}

// b~ = [sigma x - p ; z - y / rho]  (models/lu.py:30,34)
__global__ void kkt_rhs_kernel(int64_t B, int n, int m, int num_ineq, const float* p, const float* x,
                               const float* y, const float* z, float sigma, const float* scal,
                               const float* rho_rows, float* out) {
  const int N = n + m;
  const float irho_in = scal ? scal[IADMM_S_IRHO_IN] : 0.f, irho_eq = scal ? scal[IADMM_S_IRHO_EQ] : 0.f;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < B * N; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = k / N;
    const int i = (int)(k - b * N);
    if (i < n) {
      out[k] = sigma * x[b * n + i] - p[b * n + i];
    } else {
      const int j = i - n;
      const float irho = rho_rows ? 1.0f / rho_rows[b * m + j] : (j < num_ineq ? irho_in : irho_eq);
      out[k] = z[b * m + j] - irho * y[b * m + j];
    }
  }
}

// ---- The interchanges left of each block, deferred to one final pass (N <= 2048, r04) ----
// ?getrf applies block t's interchanges to the columns [0, 128 t) as soon as block t is factored;
// nothing reads those columns again before the solve, so each 128-column block j can instead take
// the composition of all later blocks' interchanges at the end, once: its rows [128 (j + 1), N)
// are read and written once (1 KB per row and block) instead of 256 rows per later block (~2x fewer
// bytes at N = 2000: 15 MB instead of 31.5 MB per instance).  The factors are bit for bit those of
// the per-block form (interchanges only move values).
//
// sigma_j[k] = the row that ends at position k of block j's columns: with pi_t the permutation of
// block t (row rowid[i] takes what row cur[i] held, build_row_perm), applying pi_{j+1}, ..., pi_{nb-1}
// in turn gives sigma_j = pi_{j+1} o sigma_{j+1}, sigma_{nb-1} = identity.  Kept with its inverse in
// LDS, each step is a sparse update over the <= 256 rows pi_t moves.
constexpr int kLeftDeferMaxN = 2048;  // rows below a block <= 1920: 15 float4 per thread at 1024 threads
__host__ __device__ inline int64_t left_sig_off(int64_t N, int64_t j) { return j * N - (int64_t)kOB * j * (j + 1) / 2; }

// one wave per instance: sigma_j on rows [128 (j + 1), N) for j = nb - 2 .. 0 into sig (per instance
// left_sig_off(N, nb - 1) ints); perm = block t's permutation at perm + t * slot + b * kPermInts
__global__ __launch_bounds__(64) void lu_left_compose_kernel(int N, int nb, int64_t slot, const int* perm, int* sig) {
  __shared__ int sg[kLeftDeferMaxN], iv[kLeftDeferMaxN];
  const int lane = threadIdx.x;
  const size_t b = blockIdx.x;
  for (int k = lane; k < N; k += 64) sg[k] = iv[k] = k;
  __syncthreads();
  int* out = sig + b * (size_t)left_sig_off(N, nb - 1);
  for (int t = nb - 1; t >= 1; --t) {
    const int* pb = perm + (size_t)t * slot + b * kPermInts;
    const int cnt = pb[4 * kPermMax];
    int kk[4], cc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int i = 64 * s + lane;
      kk[s] = i < cnt ? iv[pb[i]] : -1;
      cc[s] = i < cnt ? pb[2 * kPermMax + i] : -1;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (kk[s] >= 0) { sg[kk[s]] = cc[s]; iv[cc[s]] = kk[s]; }
    __syncthreads();
    const int r0 = kOB * t;  // sigma_{t-1}: rows [128 t, N)
    int* o = out + left_sig_off(N, t - 1);
    for (int k = r0 + lane; k < N; k += 64) o[k - r0] = sg[k];
  }
}

// rows [128 (j + 1), N) of a 16-column piece of block j take rows sigma_j (in place: every load of
// the piece, then the workgroup's barrier, then every store).  512 threads hold the piece in
// registers (15 float4 each, 96 VGPRs: two workgroups per CU, 240 KB in flight); the eight
// pieces of one (instance, block) are consecutive logical ids on one XCD, so the two 64-B halves of
// each 128-B line meet in that XCD's L2.  (r04 first form: 32-column pieces on 1024 threads, one
// workgroup per CU: 4.9 ms per factorization, ~3 TB/s.)  VEC: 16-B accesses.
template <bool VEC>
__global__ __launch_bounds__(512) void lu_left_apply_kernel(int N, int nb1, const int* sig, float* A) {
  constexpr int kLpr = VEC ? 4 : 16, kRpp = 512 / kLpr;
  constexpr int kPass = (kLeftDeferMaxN - kOB + kRpp - 1) / kRpp;
  typedef typename std::conditional<VEC, float4v, float>::type T;
  const int g = blockIdx.x, q8 = gridDim.x >> 3;  // (gridDim.x = 8 pieces x B x nb1)
  const int logical = (g & 7) * q8 + (g >> 3), piece = logical & 7, rest = logical >> 3;
  const int b = rest / nb1, j = rest % nb1;
  const int tid = threadIdx.x, rr = tid / kLpr;
  const int c = kOB * j + 16 * piece + (VEC ? 4 : 1) * (tid % kLpr);
  const int r0 = kOB * (j + 1), R = N - r0;
  const int* sg = sig + (size_t)b * left_sig_off(N, nb1) + left_sig_off(N, j);
  float* Ab = A + (size_t)b * N * N;
  T v[kPass];
#pragma unroll
  for (int p = 0; p < kPass; ++p) {
    const int src = sg[min(p * kRpp + rr, R - 1)];
    v[p] = *reinterpret_cast<const T*>(Ab + (size_t)src * N + c);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int p = 0; p < kPass; ++p) {
    const int r = p * kRpp + rr;
    if (r < R) *reinterpret_cast<T*>(Ab + (size_t)(r0 + r) * N + c) = v[p];
  }
}

}  // namespace iadmm

using namespace iadmm;

// Panels (+ in-block updates) of the 64-column half [K0, cend).
static int lu_factor_half(int64_t B, int64_t N, int K0, int cend, float* A, int* piv, int* info, hipStream_t s) {
  const bool vec = (N % 4 == 0) && aligned16(A);
  if (N <= kPanelMaxM * kLuThreads) {
    // fuse (r06): in a full 64-column half with 16-B rows the in-half updates run inside the panels
    // (lu_panel_kernel FUSE): no update launches
    const bool fuse = vec && cend - K0 == kBlk;
    for (int k0 = K0; k0 < cend; k0 += kNB) {
      const int R = (int)N - k0;
      const dim3 g((unsigned)B), t(kLuThreads);
#define IADMM_PANEL(MM)                                                                                             \
  {                                                                                                               \
    if (fuse && k0 == K0) hipLaunchKernelGGL((lu_panel_kernel<MM, kNB, kLuThreads, 0, true, 0>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info); \
    else if (fuse && k0 == K0 + kNB) hipLaunchKernelGGL((lu_panel_kernel<MM, kNB, kLuThreads, 0, true, 1>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info); \
    else if (fuse && k0 == K0 + 2 * kNB) hipLaunchKernelGGL((lu_panel_kernel<MM, kNB, kLuThreads, 0, true, 2>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info); \
    else if (fuse) hipLaunchKernelGGL((lu_panel_kernel<MM, kNB, kLuThreads, 0, true, 3>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info); \
    else hipLaunchKernelGGL((lu_panel_kernel<MM, kNB, kLuThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);         \
  }
      if (R <= kLuThreads) IADMM_PANEL(1)
      else if (R <= 2 * kLuThreads) IADMM_PANEL(2)
      else if (R <= 4 * kLuThreads) IADMM_PANEL(4)
      else if (R <= 6 * kLuThreads) IADMM_PANEL(6)
      else IADMM_PANEL(kPanelMaxM)
#undef IADMM_PANEL
      IADMM_CHECK_LAUNCH();
      const int c0 = k0 + kNB;
      if (c0 < cend && !fuse) {
        lu_update_block<kNB>(B, N, k0, cend, A, vec, s);
        IADMM_CHECK_LAUNCH();
      }
    }
  } else {  // N > 2048: 8-wide panels on 1024-thread workgroups, in registers while the panel has
            // <= kBigMaxM * kBigThreads rows, in HBM / L2 above (lu_panel_global_kernel)
    for (int k0 = K0; k0 < cend; k0 += kBigNB) {
      const int R = (int)N - k0;
      const dim3 g((unsigned)B), t(kBigThreads);
      if (R <= 2 * kBigThreads) hipLaunchKernelGGL((lu_panel_kernel<2, kBigNB, kBigThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);
      else if (R <= 4 * kBigThreads) hipLaunchKernelGGL((lu_panel_kernel<4, kBigNB, kBigThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);
      else if (R <= 8 * kBigThreads) hipLaunchKernelGGL((lu_panel_kernel<8, kBigNB, kBigThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);
      else if (R <= kBigMaxM * kBigThreads) hipLaunchKernelGGL((lu_panel_kernel<kBigMaxM, kBigNB, kBigThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);
      else hipLaunchKernelGGL((lu_panel_global_kernel<kBigNB, kBigThreads>), g, t, 0, s, (int)N, K0, k0, cend, A, piv, info);
      IADMM_CHECK_LAUNCH();
      const int c0 = k0 + kBigNB;
      if (c0 < cend) {
        lu_update_block<kBigNB>(B, N, k0, cend, A, vec, s);
        IADMM_CHECK_LAUNCH();
      }
    }
  }
  return 0;
}

// The interchanges of rows [K0, cend) (cend - K0 <= 128) on the columns [a0, a1) and [b0, b1), with
// U12 = L11^-1 A12 for the columns [b0, trsm_end) (a 64-row half only).
// (build = false: perm already holds this block's permutation.)
static int lu_swap(int64_t B, int64_t N, int K0, int cend, int a0, int a1, int b0, int b1, int trsm_end, float* A,
                   const int* piv, int* perm, hipStream_t s, bool build = true) {
  a1 = std::max(a0, a1);
  b1 = std::max(b0, b1);
  const int cols = (a1 - a0) + (b1 - b0), nbk = cend - K0;
  if (cols <= 0 || nbk <= 0) return 0;
  const dim3 grid((unsigned)B, (unsigned)((cols + 255) / 256));
  if (build && grid.y == 1 && nbk <= kBlk) {  // one workgroup per instance: built in the kernel
    if (trsm_end > b0)
      hipLaunchKernelGGL((lu_swap_kernel<kBlk, true, true>), grid, dim3(256), 0, s, (int)N, K0, nbk, a0, a1, b0, b1, trsm_end, A, perm, piv);
    else
      hipLaunchKernelGGL((lu_swap_kernel<kBlk, false, true>), grid, dim3(256), 0, s, (int)N, K0, nbk, a0, a1, b0, b1, 0, A, perm, piv);
    IADMM_CHECK_LAUNCH();
    return 0;
  }
  if (build) {
    hipLaunchKernelGGL(lu_block_perm_kernel, dim3((unsigned)B), dim3(64), 0, s, (int)N, K0, cend, piv, perm);
    IADMM_CHECK_LAUNCH();
  }
  if (trsm_end > b0)
    hipLaunchKernelGGL((lu_swap_kernel<kBlk, true>), grid, dim3(256), 0, s, (int)N, K0, nbk, a0, a1, b0, b1, trsm_end, A, perm, piv);
  else if (nbk <= kBlk)
    hipLaunchKernelGGL((lu_swap_kernel<kBlk, false>), grid, dim3(256), 0, s, (int)N, K0, nbk, a0, a1, b0, b1, 0, A, perm, piv);
  else
    hipLaunchKernelGGL((lu_swap_kernel<kPermMax, false>), grid, dim3(256), 0, s, (int)N, K0, nbk, a0, a1, b0, b1, 0, A, perm, piv);
  IADMM_CHECK_LAUNCH();
  return 0;
}

// rank-64 update A[cend.., cend..cmax) -= L21 U12 of the half [K0, cend) (lu_trail_kernel)
static int lu_rank64(int64_t B, int64_t N, int K0, int cend, int cmax, float* A, bool vec, hipStream_t s) {
  const int rest = (int)N - cend, wid = cmax - cend;
  if (rest <= 0 || wid <= 0) return 0;
  const int ntc = (wid + kTC - 1) / kTC, nrc = (rest + kTRW - 1) / kTRW;
  const dim3 grid((unsigned)(B * ntc * nrc));
  if (vec && wid <= kTC / 2)
    hipLaunchKernelGGL((lu_trail_kernel<true, 0, kTC / 2>), grid, dim3(kTrailThreads), trail_lds<kTC / 2>(), s, (int)N, K0, ntc, nrc, cmax, A);
  else if (vec) hipLaunchKernelGGL(lu_trail_kernel<true>, grid, dim3(kTrailThreads), kTrailLds, s, (int)N, K0, ntc, nrc, cmax, A);
  else hipLaunchKernelGGL(lu_trail_kernel<false>, grid, dim3(kTrailThreads), kTrailLds, s, (int)N, K0, ntc, nrc, cmax, A);
  IADMM_CHECK_LAUNCH();
  return 0;
}

// The look-ahead's streams and events (r05: a caller-owned context, iadmm_lu_ctx_create; r04 kept
// them in library statics behind a mutex, against the header's contract).  s1 (the device's highest
// priority) carries the critical path -- the block factorizations and the strips the next block
// needs -- and s2 (lowest) the rest of each trailing update, so that CUs freed by s2's workgroups go
// to s1's first.  The caller's stream forks into s1 and joins it at the end; every path out of
// lu_factor_blocks after the fork runs that join (the caller may free A, piv and ws on its stream
// as soon as the call returns).
struct iadmm_lu_ctx {
  int device = -1;
  hipStream_t s1 = nullptr, s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, ev0 = nullptr, ev1 = nullptr;
};

static int lu_linv_bufs(int64_t N);

static int lu_factor_blocks(int64_t B, int64_t N, float* A, int* piv, int* info, int* perm, int* sig,
                            float* linv, hipStream_t s0, bool gather, bool pairs, iadmm_lu_ctx* ctx) {
  hipStream_t s = s0;
  const bool vec = (N % 4 == 0) && aligned16(A);
  IADMM_ALLOW_LDS(lu_trail_kernel<true>, kTrailLds);
  IADMM_ALLOW_LDS((lu_trail_kernel<true, 0, kTC / 2>), trail_lds<kTC / 2>());
  IADMM_ALLOW_LDS(lu_trail_kernel<false>, kTrailLds);
  IADMM_ALLOW_LDS(lu_trail128_kernel<true>, kT2Lds);
  IADMM_ALLOW_LDS(lu_trail128_kernel<false>, kT2Lds);
  IADMM_ALLOW_LDS(lu_trail256_kernel<0>, kP2Lds);
  // defer: the interchanges left of each block wait for one final pass (lu_left_*_kernel); every
  // block keeps its permutation in a slot of its own until then
  const bool defer = gather && N <= kLeftDeferMaxN;
  // paired blocks (r05, the default with defer and 16-B rows; IADMM_LU_RANK128 turns them off): block t
  // (even) updates only block t + 1's columns, then one rank-256 update (lu_trail256_kernel) takes
  // everything right of block t + 1 for both -- half the A22 traffic per flop.  At B = 1024, N = 2000:
  // 75.7 ms on one stream vs 78.1 for rank-128 blocks with the look-ahead; with the look-ahead the
  // paired form took 76.9 (the rank-256 update already fills the GPU, and the panels beside it slowed
  // both), so paired factorizations run on the caller's stream (profiles/r05_lu_traces_v3.txt).
  const bool paired = pairs && defer && vec;
  const int nb = (int)((N + kOB - 1) / kOB);
  const int64_t slot = B * (int64_t)kPermInts;
  // look-ahead (with a context): block t's trailing update is two launches -- strip 0 (block t + 1's
  // own columns) on s, the other strips on a side stream -- so that block t + 1's panels, in-block
  // interchanges, in-block updates and L11^-1, which touch only block t + 1's columns, run beside the
  // rest of block t's update; block t + 1's trailing update waits for it.  The one step of block t + 1
  // that reaches further left -- its interchanges on the columns [0, P), which hold block t's L21 that
  // the side launch still reads -- waits for it too (N > 2048, r05; N <= 2048 defers that step to the
  // end).  L11^-1 and (without defer) the block permutation alternate between two buffers.
  // (without a context, or with the interchanges as a pass of their own (gather = false), everything
  // runs in order on the caller's stream)
  iadmm_lu_ctx* side = gather && !paired ? ctx : nullptr;
  // Under stream capture the critical path stays on the caller's (capturing) stream and the side
  // strips fork from it directly (r06).  The eager hop s0 -> s1 -> s2 is a fork from a stream that
  // joined the capture through another forked stream, and the HIP runtime python processes load --
  // PyTorch's bundled libamdhip64 (ROCm 7.0.2), which this library binds to by soname -- crashes in
  // hipStreamEndCapture on exactly that shape (tools/capture_probe.hip variant 2; variants 1, 9, 10,
  // forks from the capture's origin only, capture and replay; the system HIP 7.2 runtime takes all of
  // them: profiles/r06_capture_probe.txt).  r05 ran the whole factorization on one stream under
  // capture instead; the captured graph now has the eager schedule's concurrency.  (Stream
  // priorities do not carry into a graph, so s1's role is moot there.)
  bool capturing = false;
  if (side) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    IADMM_HIP_RC(hipStreamIsCapturing(s0, &cs));
    capturing = cs != hipStreamCaptureStatusNone;
  }
  if (side && !capturing) {  // (nothing is enqueued on s1 before both calls succeed: a failure returns unforked)
    IADMM_HIP_RC(hipEventRecord(side->ev0, s0));
    IADMM_HIP_RC(hipStreamWaitEvent(side->s1, side->ev0, 0));
    s = side->s1;
  }
  bool pending = false;  // a side launch not yet joined
  int rc = 0;
  // after the fork no error may return early: record it, leave the loop, and still join below
#define LU_TRY(call)                              \
  {                                               \
    const hipError_t e_ = (call);                 \
    if (e_ != hipSuccess) { rc = (int)e_; break; } \
  }
#define LU_TRY_LAUNCH() LU_TRY(hipGetLastError())
  for (int P = 0; P < N && !rc; P += kOB) {
    const int n_ = (int)N;
    const int c1 = std::min(n_, P + kBlk), c2 = std::min(n_, P + kOB);
    int* pm = defer ? perm + (P / kOB) * slot : (side ? perm + ((P / kOB) & 1) * slot : perm);
    // first half: factor; its interchanges and U12 on the second half's columns only, then the second
    // half's rank-64 update
    rc = lu_factor_half(B, N, P, c1, A, piv, info, s);
    if (!rc && c1 < n_) rc = lu_swap(B, N, P, c1, 0, 0, c1, c2, c2, A, piv, pm, s);
    if (!rc) rc = lu_rank64(B, N, P, c1, c2, A, vec, s);
    // second half: factor; its interchanges on the first half's columns
    if (!rc && c1 < n_) rc = lu_factor_half(B, N, c1, c2, A, piv, info, s);
    if (!rc && c1 < n_) rc = lu_swap(B, N, c1, c2, P, c1, 0, 0, 0, A, piv, pm, s);
    // the whole block's interchanges composed into one row permutation: applied to the columns right
    // of the block inside lu_trail128_kernel (gathered loads) -- or here (gather = false: N above the
    // trailing kernel's LDS tables), then an interchange-free trailing update -- and to the columns
    // left of it here, or at the end (defer)
    if (rc) break;
    // (defer: nothing to swap here, and L11^-1's kernel builds the permutation beside the substitution)
    const bool perm_in_linv = defer && c2 < n_;
    if (!perm_in_linv) {
      hipLaunchKernelGGL(lu_block_perm_kernel, dim3((unsigned)B), dim3(64), 0, s, (int)N, P, c2, piv, pm);
      LU_TRY_LAUNCH();
    }
    if (!defer && pending) {  // block t - 1's other strips read its L21, which the left interchanges move
      LU_TRY(hipStreamWaitEvent(s, side->join, 0));
      pending = false;
    }
    rc = lu_swap(B, N, P, c2, 0, defer ? 0 : P, gather ? 0 : c2, gather ? 0 : n_, 0, A, piv, pm, s, false);
    if (rc || c2 >= n_) break;
    // U12 = L11^-1 A12 and the rank-128 update of everything right of the block
    const int t = P / kOB;
    const int nbuf = lu_linv_bufs(N);
    float* lv = linv + (side || paired ? (t % nbuf) : 0) * B * (int64_t)kLinvFloats;
    hipLaunchKernelGGL(lu_linv_kernel, dim3((unsigned)B), dim3(kOB + 64), 0, s, (int)N, P, A, lv, piv,
                       perm_in_linv ? pm : nullptr, c2);
    LU_TRY_LAUNCH();
    // pairs: block t even with columns beyond block t + 1 updates only block t + 1's columns (strip
    // 0); block t + 1 then updates everything right of it for both blocks at rank 256
    const bool first = paired && (t % 2 == 0) && P + kR2 < n_;
    const bool second = paired && (t % 2 == 1);  // (t - 1 was a first: its P + 256 = c2 < N here)
    const int Pp = second ? P - kOB : P;      // the update's own P (the pair's first row)
    const int ntc = ((int)N - c2 + kT2C - 1) / kT2C;
    const int* gp = gather ? pm : nullptr;
    const float* lv0 = linv + ((t + nbuf - 1) % nbuf) * B * (int64_t)kLinvFloats;  // block t - 1's (pairs)
    auto trail = [&](hipStream_t st, int tc0, int cnt) {
      const dim3 grid((unsigned)(B * cnt));
      if (second) hipLaunchKernelGGL(lu_trail256_kernel<0>, grid, dim3(kD2Threads), kP2Lds, st, (int)N, Pp, cnt, tc0, A, lv0, lv, pm - slot, pm);
      else if (vec) hipLaunchKernelGGL(lu_trail128_kernel<true>, grid, dim3(kT2Threads), kT2Lds, st, (int)N, P, cnt, tc0, A, lv, gp);
      else hipLaunchKernelGGL(lu_trail128_kernel<false>, grid, dim3(kT2Threads), kT2Lds, st, (int)N, P, cnt, tc0, A, lv, gp);
    };
    if (first) {  // strip 0 only, in order on s (the previous pair's far strips joined first)
      if (pending) {
        LU_TRY(hipStreamWaitEvent(s, side->join, 0));
        pending = false;
      }
      trail(s, 0, 1);
      LU_TRY_LAUNCH();
      continue;
    }
    if (!side) {
      trail(s, 0, ntc);
      LU_TRY_LAUNCH();
      continue;
    }
    if (pending) {  // block t - 1's other strips
      LU_TRY(hipStreamWaitEvent(s, side->join, 0));
      pending = false;
    }
    if (ntc > 1) {
      LU_TRY(hipEventRecord(side->fork, s));
      LU_TRY(hipStreamWaitEvent(side->s2, side->fork, 0));
      trail(side->s2, 1, ntc - 1);
      const hipError_t e = hipGetLastError();
      // (join even after a failed launch: whatever reached s2 is ordered before the caller's stream)
      LU_TRY(hipEventRecord(side->join, side->s2));
      pending = true;
      LU_TRY(e);
    }
    trail(s, 0, 1);
    LU_TRY_LAUNCH();
  }
#undef LU_TRY
#undef LU_TRY_LAUNCH
  auto keep = [&rc](hipError_t e) {  // the first error wins
    if (e != hipSuccess && !rc) rc = (int)e;
  };
  if (pending && !rc && hipStreamWaitEvent(s, side->join, 0) == hipSuccess) pending = false;
  if (!rc && defer && nb > 1) {
    hipLaunchKernelGGL(lu_left_compose_kernel, dim3((unsigned)B), dim3(64), 0, s, (int)N, nb, slot, perm, sig);
    keep(hipGetLastError());
    if (!rc) {
      const dim3 grid((unsigned)(B * 8 * (nb - 1)));
      if (vec) hipLaunchKernelGGL(lu_left_apply_kernel<true>, grid, dim3(512), 0, s, (int)N, nb - 1, sig, A);
      else hipLaunchKernelGGL(lu_left_apply_kernel<false>, grid, dim3(512), 0, s, (int)N, nb - 1, sig, A);
      keep(hipGetLastError());
    }
  }
  if (side) {  // the caller's stream joins s1 -- and s2 directly if s1 has not -- on every path after the fork
    if (s != s0) {
      const hipError_t e1 = hipEventRecord(side->ev1, s);
      keep(e1 == hipSuccess ? hipStreamWaitEvent(s0, side->ev1, 0) : e1);
    }
    if (pending) keep(hipStreamWaitEvent(s0, side->join, 0));
  }
  return rc;
}

// ---- Solve with x in HBM (N above the LDS-resident lu_solve_kernel's limit, r04) ----
// P b, then forward (unit L) and backward (U) substitution in 64-row blocks, right-looking: per
// block one launch solves the diagonal block (one wave per instance, the block in LDS) and one
// launch subtracts its contribution from every remaining row (lu_solve_gemv_kernel: 64 rows per
// workgroup, 16 lanes per row, all workgroups of the grid streaming the block column).  Launch-bound
// (four launches per block pair), but every CU streams the factors, which one workgroup per
// instance could not at the batch sizes such N leaves room for.

// P b: each 64-row block's interchanges composed (build_row_perm) and applied with every load
// before every store; one wave per instance walks the blocks in order.
__global__ __launch_bounds__(64) void lu_solve_perm_kernel(int N, const int* piv, float* X) {
  __shared__ int pvs[kSolveBlk], prow[2 * kSolveBlk], pcur[2 * kSolveBlk], pcnt[1];
  const int lane = threadIdx.x;
  const size_t b = blockIdx.x;
  float* x = X + b * N;
  for (int k0 = 0; k0 < N; k0 += kSolveBlk) {
    const int nbk = min(kSolveBlk, N - k0);
    if (lane < nbk) pvs[lane] = piv[b * N + k0 + lane] - 1;
    __syncthreads();
    build_row_perm(pvs, k0, nbk, prow, pcur, pcnt);
    const int cnt = *pcnt;
    const float v0 = x[pcur[min(lane, cnt - 1)]], v1 = x[pcur[min(lane + 64, cnt - 1)]];
    if (lane < cnt) x[prow[lane]] = v0;
    if (lane + 64 < cnt) x[prow[lane + 64]] = v1;
    __syncthreads();  // (the stores ordered before the next block's loads; LDS tables reused)
  }
}

// x[k0, k1) <- (unit lower | upper) triangle of the diagonal block \ x[k0, k1); one wave per instance.
template <bool UPPER>
__global__ __launch_bounds__(64) void lu_solve_tri_kernel(int N, const float* LU, float* X, int k0) {
  __shared__ float D[kSolveBlk][kSolveBlk + 1];
  const int lane = threadIdx.x;
  const size_t b = blockIdx.x;
  const float* M = LU + b * (size_t)N * N;
  float* x = X + b * N;
  const int nbk = min(kSolveBlk, N - k0);
  const int c = min(lane, nbk - 1);
  float d[kSolveBlk];
#pragma unroll
  for (int r = 0; r < kSolveBlk; ++r) d[r] = M[(size_t)(k0 + min(r, nbk - 1)) * N + k0 + c];  // all in flight
#pragma unroll
  for (int r = 0; r < kSolveBlk; ++r) D[r][lane] = d[r];
  __syncthreads();
  float v = lane < nbk ? x[k0 + lane] : 0.f;
  if (!UPPER) {
    for (int j = 0; j < nbk; ++j) {
      const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
      if (lane > j && lane < nbk) v = fmaf(-D[lane][j], xj, v);
    }
  } else {
    for (int j = nbk - 1; j >= 0; --j) {
      const float vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j)) / D[j][j];
      if (lane == j) v = vj;
      if (lane < j) v = fmaf(-D[lane][j], vj, v);
    }
  }
  if (lane < nbk) x[k0 + lane] = v;
}

// x[r] -= M[r, k0:k1) . x[k0:k1) for r in [r0, r1): 64 rows per workgroup (grid (B, row blocks)),
// 4 rows per wave at a time, lane (row, q = lane & 15) holding columns 4q .. 4q + 3 of the block.
template <bool VEC>
__global__ __launch_bounds__(256) void lu_solve_gemv_kernel(int N, const float* LU, float* X, int k0, int r0, int r1) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane & 15;
  const size_t b = blockIdx.x;
  const float* M = LU + b * (size_t)N * N;
  float* x = X + b * N;
  const int nbk = min(kSolveBlk, N - k0);
  float xv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) xv[e] = 4 * q + e < nbk ? x[k0 + 4 * q + e] : 0.f;
  const int rbase = r0 + blockIdx.y * 64 + wave * 16;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int r = rbase + 4 * g + (lane >> 4);
    const int rr = min(r, r1 - 1);
    const float* row = M + (size_t)rr * N + k0 + 4 * q;
    float a[4];
    if (VEC && 4 * q + 3 < nbk) {
      const float4 t = *reinterpret_cast<const float4*>(row);
      a[0] = t.x; a[1] = t.y; a[2] = t.z; a[3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = 4 * q + e < nbk ? row[min(e, nbk - 1 - 4 * q)] : 0.f;
    }
    float sum = fmaf(a[3], xv[3], fmaf(a[2], xv[2], fmaf(a[1], xv[1], a[0] * xv[0])));
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) sum += __shfl_xor(sum, off, 16);
    if (q == 0 && r < r1) x[r] -= sum;
  }
}

static int lu_solve_hbm(int64_t B, int64_t N, const float* LU, const int* piv, float* x, hipStream_t s) {
  const bool vec = N % 4 == 0 && aligned16(LU);
  hipLaunchKernelGGL(lu_solve_perm_kernel, dim3((unsigned)B), dim3(64), 0, s, (int)N, piv, x);
  IADMM_CHECK_LAUNCH();
  const int nblk = (int)((N + kSolveBlk - 1) / kSolveBlk);
  for (int bb = 0; bb < nblk; ++bb) {  // forward, unit L
    const int k0 = bb * kSolveBlk, k1 = std::min((int)N, k0 + kSolveBlk);
    hipLaunchKernelGGL(lu_solve_tri_kernel<false>, dim3((unsigned)B), dim3(64), 0, s, (int)N, LU, x, k0);
    IADMM_CHECK_LAUNCH();
    if (k1 < N) {
      const dim3 g((unsigned)B, (unsigned)((N - k1 + 63) / 64));
      if (vec) hipLaunchKernelGGL(lu_solve_gemv_kernel<true>, g, dim3(256), 0, s, (int)N, LU, x, k0, k1, (int)N);
      else hipLaunchKernelGGL(lu_solve_gemv_kernel<false>, g, dim3(256), 0, s, (int)N, LU, x, k0, k1, (int)N);
      IADMM_CHECK_LAUNCH();
    }
  }
  for (int bb = nblk - 1; bb >= 0; --bb) {  // backward, U
    const int k0 = bb * kSolveBlk;
    hipLaunchKernelGGL(lu_solve_tri_kernel<true>, dim3((unsigned)B), dim3(64), 0, s, (int)N, LU, x, k0);
    IADMM_CHECK_LAUNCH();
    if (k0 > 0) {
      const dim3 g((unsigned)B, (unsigned)((k0 + 63) / 64));
      if (vec) hipLaunchKernelGGL(lu_solve_gemv_kernel<true>, g, dim3(256), 0, s, (int)N, LU, x, k0, 0, k0);
      else hipLaunchKernelGGL(lu_solve_gemv_kernel<false>, g, dim3(256), 0, s, (int)N, LU, x, k0, 0, k0);
      IADMM_CHECK_LAUNCH();
    }
  }
  return 0;
}

// workspace: per-instance block permutations (kPermInts ints; N <= kLeftDeferMaxN: one slot per
// 128-column block, then the deferred left interchanges' sigma tables; up to kLuMaxN two alternating
// slots), then the 128 x 128 two-level L11^-1 of the current outer block (two alternating buffers up
// to kLuMaxN; each part 16-B aligned)
static int64_t al16(int64_t n) { return (n + 15) / 16 * 16; }
static int64_t lu_nb(int64_t N) { return (N + kOB - 1) / kOB; }
static int64_t lu_perm_bytes(int64_t B, int64_t N) {  // (two alternating slots for the look-ahead)
  return al16(B * (int64_t)kPermInts * (N <= kLeftDeferMaxN ? lu_nb(N) : (N <= kLuMaxN ? 2 : 1)) * (int64_t)sizeof(int));
}
static int64_t lu_sig_bytes(int64_t B, int64_t N) {
  return N <= kLeftDeferMaxN ? al16(B * left_sig_off(N, lu_nb(N) - 1) * (int64_t)sizeof(int)) : 0;
}
// Two alternating L11^-1 buffers: the look-ahead factors block t + 1 (writing its buffer) while block
// t's update still reads the other; a paired update reads blocks t and t + 1's (both), and block t + 2
// rewrites block t's only after that update, in order on the same stream (a batch split gives each half
// its own workspace).  (r05 sized four for the paired form; ADVICE r05: nothing read them concurrently.)
static int lu_linv_bufs(int64_t N) {
  return N <= kLuMaxN ? 2 : 1;
}
static int64_t lu_ws_bytes(int64_t B, int64_t N) {
  return lu_perm_bytes(B, N) + lu_sig_bytes(B, N) +
         lu_linv_bufs(N) * B * (int64_t)kLinvFloats * (int64_t)sizeof(float);
}

// (+ 64 B: the two half-batch workspaces of a split factorization round up separately)
extern "C" int64_t iadmm_lu_factor_ws_bytes(int64_t B, int64_t N) {
  if (B <= 0 || N <= 0) return 0;
  return lu_ws_bytes(B, N) + 64;
}

extern "C" int iadmm_lu_ctx_create(iadmm_lu_ctx** out) {
  if (!out) return IADMM_E_ARG;
  *out = nullptr;
  iadmm_lu_ctx* c = new (std::nothrow) iadmm_lu_ctx();
  if (!c) return (int)hipErrorOutOfMemory;
  hipError_t e = hipGetDevice(&c->device);
  int least = 0, greatest = 0;
  if (e == hipSuccess && hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->s1, hipStreamNonBlocking, greatest);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->s2, hipStreamNonBlocking, least);
  hipEvent_t* evs[4] = {&c->fork, &c->join, &c->ev0, &c->ev1};
  for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(evs[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    (void)iadmm_lu_ctx_destroy(c);
    return (int)e;
  }
  *out = c;
  return 0;
}

extern "C" int iadmm_lu_ctx_destroy(iadmm_lu_ctx* c) {
  if (!c) return 0;
  hipError_t first = hipSuccess;
  auto keep = [&first](hipError_t e) { if (first == hipSuccess) first = e; };
  for (hipEvent_t ev : {c->fork, c->join, c->ev0, c->ev1})
    if (ev) keep(hipEventDestroy(ev));
  for (hipStream_t st : {c->s1, c->s2})
    if (st) keep(hipStreamDestroy(st));  // (returns once the stream's work is done)
  delete c;
  return (int)first;
}

extern "C" int iadmm_lu_factor_ex(int64_t B, int64_t N, float* A, int* piv, int* info, void* ws, int64_t ws_bytes,
                                  iadmm_lu_ctx* ctx, int flags, void* stream) {
  if (B <= 0 || N <= 0 || !A || !piv || !info || !ws) return IADMM_E_ARG;
  if (ws_bytes < lu_ws_bytes(B, N) + 64) return IADMM_E_ARG;  // (= iadmm_lu_factor_ws_bytes)
  if (flags & ~(IADMM_LU_FORCE_HBM | IADMM_LU_PAIRS | IADMM_LU_RANK128)) return IADMM_E_ARG;
  if (!aligned16(ws)) return IADMM_E_ALIGN;
  if (N > kLuMaxHbmN || B > 0x7fffffff) return IADMM_E_SIZE;
  const int64_t ntc_max = (N + kTC - 1) / kTC, nrc_max = (N + kTRW - 1) / kTRW;
  if (B * ntc_max * nrc_max > 0x7fffffff) return IADMM_E_SIZE;
  if (ctx) {  // a context belongs to the device it was made on
    int dev = -1;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev != ctx->device) return IADMM_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(lu_info_zero_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B, info);
  IADMM_CHECK_LAUNCH();
  const bool gather = N <= kLuMaxN && !(flags & IADMM_LU_FORCE_HBM);
  const bool pairs = !(flags & IADMM_LU_RANK128);
  auto run = [&](int64_t b0, int64_t nb, char* w, hipStream_t st, iadmm_lu_ctx* c) {
    int* perm = reinterpret_cast<int*>(w);
    int* sig = reinterpret_cast<int*>(w + lu_perm_bytes(nb, N));
    float* linv = reinterpret_cast<float*>(w + lu_perm_bytes(nb, N) + lu_sig_bytes(nb, N));
    return lu_factor_blocks(nb, N, A + b0 * N * N, piv + b0 * N, info + b0, perm, sig, linv, st, gather, pairs, c);
  };
  // Batch split (r05): the paired-block form runs on one stream (no look-ahead), so with a context and a
  // batch of at least two instances per CU the two halves are factored concurrently on the context's
  // two streams -- the instances share nothing, so the factors are bit for bit those of one call, and
  // one half's latency-bound panel steps overlap the other half's updates (B = 1024, N = 2000: 75.8 ->
  // 74.1 ms, profiles/r05_lu_split_ab.txt; four parts: 78.7).  Both halves fork from the caller's stream
  // by one event, which a stream capture takes as well (tools/capture_probe.hip variant 9; r06 -- r05
  // kept captured factorizations on one stream).
  const bool split = ctx && pairs && gather && N <= kLeftDeferMaxN && N % 4 == 0 && aligned16(A) && B >= 512 &&
                     ws_bytes >= lu_ws_bytes(B / 2, N) + lu_ws_bytes(B - B / 2, N);
  if (!split) return run(0, B, static_cast<char*>(ws), s, ctx);
  const int64_t B0 = B / 2, B1 = B - B0;
  char* w1 = static_cast<char*>(ws) + lu_ws_bytes(B0, N);  // (16-B multiple)
  IADMM_HIP_RC(hipEventRecord(ctx->ev0, s));
  IADMM_HIP_RC(hipStreamWaitEvent(ctx->s1, ctx->ev0, 0));
  IADMM_HIP_RC(hipStreamWaitEvent(ctx->s2, ctx->ev0, 0));
  // from here on both streams are joined back into s whatever fails
  int rc = run(0, B0, static_cast<char*>(ws), ctx->s1, nullptr);
  const int rc1 = run(B0, B1, w1, ctx->s2, nullptr);
  if (!rc) rc = rc1;
  hipError_t e = hipEventRecord(ctx->ev1, ctx->s1);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, ctx->ev1, 0);
  if (e != hipSuccess && !rc) rc = (int)e;
  e = hipEventRecord(ctx->join, ctx->s2);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, ctx->join, 0);
  if (e != hipSuccess && !rc) rc = (int)e;
  return rc;
}

extern "C" int iadmm_lu_factor(int64_t B, int64_t N, float* A, int* piv, int* info, void* ws, int64_t ws_bytes,
                               void* stream) {
  return iadmm_lu_factor_ex(B, N, A, piv, info, ws, ws_bytes, nullptr, 0, stream);
}

extern "C" int iadmm_lu_solve_ex(int64_t B, int64_t N, const float* LU, const int* piv, float* x, int flags,
                                 void* stream) {
  if (B <= 0 || N <= 0 || !LU || !piv || !x) return IADMM_E_ARG;
  if (flags & ~IADMM_LU_FORCE_HBM) return IADMM_E_ARG;
  const size_t lds = ((size_t)N + kSolveBlk + kSolveBlk * kDS) * sizeof(float);
  if (N > kLuMaxHbmN || B > 0x7fffffff || B * ((N + 63) / 64) > 0x7fffffff) return IADMM_E_SIZE;
  // gfx950: 160 KiB of LDS per workgroup; x beyond it lives in HBM
  if (lds > 160 * 1024 || (flags & IADMM_LU_FORCE_HBM)) return lu_solve_hbm(B, N, LU, piv, x, (hipStream_t)stream);
  IADMM_ALLOW_LDS(lu_solve_kernel<true>, lds);
  IADMM_ALLOW_LDS(lu_solve_kernel<false>, lds);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  IADMM_ALLOW_LDS((lu_solve_kernel<true, 512>), lds);
  IADMM_ALLOW_LDS((lu_solve_kernel<true, 1024>), lds);
  if (N % 4 == 0 && aligned16(LU) && B <= cus)
    hipLaunchKernelGGL((lu_solve_kernel<true, 1024>), dim3((unsigned)B), dim3(1024), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  else if (N % 4 == 0 && aligned16(LU) && B <= 2 * cus)
    hipLaunchKernelGGL((lu_solve_kernel<true, 512>), dim3((unsigned)B), dim3(512), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  else if (N % 4 == 0 && aligned16(LU))
    hipLaunchKernelGGL(lu_solve_kernel<true>, dim3((unsigned)B), dim3(kSolveThreads), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  else
    hipLaunchKernelGGL(lu_solve_kernel<false>, dim3((unsigned)B), dim3(kSolveThreads), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_lu_solve(int64_t B, int64_t N, const float* LU, const int* piv, float* x, void* stream) {
  return iadmm_lu_solve_ex(B, N, LU, piv, x, 0, stream);
}

extern "C" int iadmm_kkt_rhs(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* p,
                             const float* x, const float* y, const float* z, float sigma,
                             const float* scal, const float* rho_rows, float* out, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !p || !x || !out || (m > 0 && (!y || !z))) return IADMM_E_ARG;
  if (m > 0 && !scal && !rho_rows) return IADMM_E_ARG;
  const int64_t tot = B * (n + m);
  const int64_t blocks = (tot + 255) / 256;
  hipLaunchKernelGGL(kkt_rhs_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)n, (int)m, (int)num_ineq, p, x, y, z, sigma, scal,
                     rho_rows, out);
  IADMM_CHECK_LAUNCH();
  return 0;
}
