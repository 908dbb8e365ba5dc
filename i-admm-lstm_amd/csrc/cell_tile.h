// The K-loop of the fused LSTM-cell GEMM, shared by the forward kernel (lstm.hip) and the
// recompute in the training backward (train.hip).  See lstm.hip for the tiling.
#pragma once
#include "common.h"
#include <type_traits>

namespace iadmm {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kJT = 32;          // hidden units per workgroup
constexpr int kRows = 256;       // data rows per workgroup
constexpr int kBK = 32;          // K chunk
constexpr int kLD = kBK + 4;     // padded LDS row (floats)
constexpr int kWxF = 16;         // packed per-unit fields: Wi0 Wi1 bi Wf0 Wf1 bf Wo0 Wo1 bo Wu0 Wu1 bu Wh

struct CellArgsT {
  int64_t M;
  int h, njt, nkc32;
  const float *H, *C, *xv, *g, *Upk, *Wx;
  float *Hn, *Cn, *part;
  int pgroup;  // panels per tile group of cell_tile_of_block_grouped (0 or 1: hidden tile fastest)
};

// XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of
// logical tiles with the hidden tile fastest, so an H panel is reused from that XCD's L2.
IADMM_DEV void cell_tile_of_block(int njt, int& jt, int& rt) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  jt = logical % njt;
  rt = logical / njt;
}

// Grouped variant: the logical tiles (same XCD-contiguous ranges as above) are walked in groups of
// pg row panels x all njt hidden tiles, hidden tile SLOWEST inside a group: the pg workgroups of
// one hidden tile are dispatched back to back, so they stream the same weight slice at the same K
// position (one L2 fill serves pg workgroups), while a panel's njt workgroups stay within one
// group (pg * njt consecutive dispatches).  pg <= 1 is cell_tile_of_block.
IADMM_DEV void cell_tile_of_block_grouped(int njt, int64_t nrt, int pg, int& jt, int& rt) {
  if (pg <= 1) {
    cell_tile_of_block(njt, jt, rt);
    return;
  }
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int S = pg * njt;
  const int st = logical / S, r = logical - st * S;
  const int p0 = st * pg;
  const int pl = (int)(nrt - p0 < pg ? nrt - p0 : pg);
  jt = r / pl;
  rt = p0 + (r - jt * pl);
}

// acc[g][r] (4 gates x 2 row blocks of 32x32) = U_g[:, jt*32 .. +32]^T . H[rbase + wave*64 + r*32 ..]^T
// NW waves per workgroup (64*NW data rows).  PRIO: 0 none; 1 s_setprio(1) around each MFMA
// cluster; 2 (NW = 8) static priority 1 for waves 4-7 (cdna_hip_programming.md T5).
template <bool VEC, int NW = 4, int PRIO = 0, bool BUF = false>
IADMM_DEV void cell_mainloop(const float* __restrict__ H, int64_t M, int h, int nkc,
                             const float* __restrict__ Ubase, int64_t rbase, float* sA, float* sB,
                             floatx16 (&acc)[4][2], int tid, int wave, int jl, int hf) {
  constexpr int NT = 64 * NW;
  constexpr int A4 = 128 * kBK / 4 / NT;  // weight float4 per thread: 4 (NW 4) or 2 (NW 8)
  static_assert(A4 == 4 || A4 == 2, "NW must be 4 or 8");
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;
  if constexpr (PRIO == 2) {
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  // Staging registers as named scalars (an array here was turned into an LDS/scratch alloca
  // by the compiler, which then waited for each global load right after issuing it).
  float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7;
  // BUF: the H panel through a buffer descriptor whose range ends at the last valid row, so a
  // row past M (and a k past h, offset forced out of range) reads 0 without a branch: no
  // predicated load, no phi, no early vmcnt wait.
  const int64_t nvalid = (M - rbase) < NT ? (M - rbase) : NT;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(H + rbase * h), 0, (int)(nvalid * h * 4), 0x00020000);
  auto ldB = [&](int kc, int i) -> float4 {
    const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
    const int64_t R = rbase + row;
    const int k = kc * kBK + c4 * 4;
    if constexpr (BUF) {
      static_assert(VEC, "BUF needs h % 4 == 0");
      const unsigned off = k < h ? (unsigned)(row * h + k) * 4u : 0x80000000u;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(hrs, off, 0, 0);
      return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
    } else if constexpr (VEC) {
      return (R < M && k < h) ? *reinterpret_cast<const float4*>(H + R * h + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      float4 t;
#pragma unroll
      for (int e = 0; e < 4; ++e) set4(t, e, (R < M && k + e < h) ? H[R * h + k + e] : 0.f);
      return t;
    }
  };
  auto gload = [&](int kc) {
    const float4* Ac = reinterpret_cast<const float4*>(Ubase + (int64_t)kc * 128 * kBK);
    ra0 = Ac[tid];
    ra1 = Ac[tid + NT];
    if constexpr (A4 == 4) {
      ra2 = Ac[tid + 2 * NT];
      ra3 = Ac[tid + 3 * NT];
    }
    rb0 = ldB(kc, 0); rb1 = ldB(kc, 1); rb2 = ldB(kc, 2); rb3 = ldB(kc, 3);
    rb4 = ldB(kc, 4); rb5 = ldB(kc, 5); rb6 = ldB(kc, 6); rb7 = ldB(kc, 7);
  };
  auto st = [&](float* sm, int i, const float4& v) {
    const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
    *reinterpret_cast<float4*>(&sm[row * kLD + c4 * 4]) = v;
  };

  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
    st(sA, 0, ra0); st(sA, 1, ra1);
    if constexpr (A4 == 4) { st(sA, 2, ra2); st(sA, 3, ra3); }
    st(sB, 0, rb0); st(sB, 1, rb1); st(sB, 2, rb2); st(sB, 3, rb3);
    st(sB, 4, rb4); st(sB, 5, rb5); st(sB, 6, rb6); st(sB, 7, rb7);
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int G = 0; G < kBK / 8; ++G) {
      float4 af[4], bf[2];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        af[g] = *reinterpret_cast<const float4*>(&sA[(g * 32 + jl) * kLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bf[r] = *reinterpret_cast<const float4*>(&sB[(wave * 64 + r * 32 + jl) * kLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(af[g], s), get4(bf[r], s),
                                                             acc[g][r], 0, 0, 0);
    }
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
}


// ---- LDS-DMA main loop (gfx950 buffer_load_dwordx4 ... lds): same products, same accumulation
// order as cell_mainloop (k = 32*kc32 + 8*G + 4*hf + s), so the result is bitwise identical.
//
// K is staged in 16-deep chunks through a 3-stage LDS ring filled directly by LDS-DMA (no staging
// registers, no ds_write pass): per chunk and wave, 2 pieces of the weight tile + 4 pieces of the
// H panel (1 KiB each).  Every LDS row is 16 floats (64 B) with its four 16-B slots XOR-swizzled
// by (row >> 2) & 3 on the SOURCE address (the DMA image is lane-linear), which makes the
// fragment ds_read_b128 conflict-free.  One barrier per chunk, placed between the two 8-deep
// halves: before it, each wave waits only for its own pieces of chunk kc+1 (counted vmcnt, chunk
// kc+2 never in flight yet); after it, chunk kc+2 is issued into the stage chunk kc-1 used and the
// first fragments of chunk kc+1 are read while the second half of chunk kc runs on the MFMA pipe.
// Fragments are double-buffered in registers so no MFMA waits on an LDS read it just issued.
constexpr int kBKd = 16;                          // K chunk of the DMA ring
constexpr int kStages = 3;
constexpr int kStageA = 128 * kBKd;               // floats: 4 gates x 32 units x 16 k
constexpr int kStageB = 256 * kBKd;               // floats: 256 rows x 16 k
constexpr int kRingFloats = kStages * (kStageA + kStageB);  // 73728 B

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
IADMM_DEV void vm_wait() {  // s_waitcnt vmcnt(N), other counters untouched (gfx9 encoding)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// acc[g][r] += A[g*32 + .., k] . B[wave*64 + r*32 + .., k] over k < K, through the LDS ring.
//   B: row-major panel (row stride ldb floats) starting at the workgroup's first row; rows past
//      nb_valid and k past K read as zero (buffer range check / out-of-range offset).
//   A: NA*32 rows (NA = 4: the cell's 4 gates x 32 units; 5: 160-row GEMM tiles).  A_PACKED: the
//      fp32 32-deep packing [ceil(K/32)][NA*32][32] (lstm_pack_kernel / gemm_pack_a; Abase = the
//      tile's block, zero-padded); otherwise row-major, row stride lda, rows past na_valid and k
//      past K zero.
// before_last() runs once, just before the last chunk's MFMAs (e.g. to prefetch epilogue operands
// behind them).
template <bool A_PACKED, int NA = 4, class BeforeLast>
IADMM_DEV void mainloop_dma(const float* __restrict__ Abase, int na_valid, int lda,
                            const float* __restrict__ Bbase, int64_t nb_valid, int ldb, int K,
                            float* ring, floatx16 (&acc)[NA][2], int tid, int wave, int jl, int hf,
                            BeforeLast&& before_last) {
  static_assert(NA == 4 || NA == 5, "A tile = 4 or 5 blocks of 32 rows");
  constexpr int AROWS = NA * 32;
  constexpr int STA = AROWS * kBKd;                 // floats of the A part of a stage
  constexpr int ST = STA + kStageB;                 // floats per stage
  constexpr int NPA = NA * 2;                       // A pieces per chunk (16 rows each)
  constexpr int APW = (NPA + 3) / 4;                // A pieces per wave (the last may be a dummy)
#pragma unroll
  for (int g = 0; g < NA; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;

  const int lane = tid & 63;
  const int nk = (K + kBKd - 1) / kBKd;
  const int nkc32 = (K + kBK - 1) / kBK;
  const int64_t nbv = nb_valid < 256 ? nb_valid : 256;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(Bbase), 0, (int)(nbv * ldb * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(Abase), 0,
      A_PACKED ? nkc32 * AROWS * kBK * 4 : (na_valid < AROWS ? na_valid : AROWS) * lda * 4, 0x00020000);

  // Per-lane source offsets of this wave's pieces (piece = 16 LDS rows x 4 slots).  A piece p is
  // issued by wave p % 4; a wave with fewer real pieces issues an out-of-range dummy into the
  // scratch KiB after the ring (so every wave runs the same instruction stream).
  const int prow = lane >> 2, pslot = lane & 3;
  unsigned aoff[APW];
  int ak4[APW];
  int bk4[4];
  unsigned boff[4];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int p = wave + 4 * i;
    const int row = p * 16 + prow;                          // g*32 + jj
    const int c = pslot ^ ((row >> 2) & 3);
    ak4[i] = p < NPA ? c * 4 : (1 << 30);                   // dummy: every k out of range
    aoff[i] = A_PACKED ? (unsigned)(row * kBK + c * 4) * 4u    // + kc32*16 KiB + half*64 B
                       : (unsigned)(row * lda + c * 4) * 4u;   // + kc*64 B
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 16 + prow;
    const int c = pslot ^ ((row >> 2) & 3);
    bk4[i] = c * 4;
    boff[i] = (unsigned)(row * ldb + c * 4) * 4u;            // + kc*64 B
  }
  auto issue = [&](int kc) {
    const int st = kc % kStages;
    float* sa = ring + st * ST;
    float* sb = sa + STA;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int p = wave + 4 * i;
      unsigned o;
      if constexpr (A_PACKED) {
        o = (NPA % 4 == 0 || p < NPA) ? aoff[i] + (unsigned)((kc >> 1) * AROWS * kBK + (kc & 1) * kBKd) * 4u
                                      : 0x80000000u;
      } else {
        o = (kc * kBKd + ak4[i] < K) ? aoff[i] + (unsigned)(kc * kBKd * 4) : 0x80000000u;
      }
      float* dst = (NPA % 4 == 0 || p < NPA) ? sa + p * 256 : ring + kStages * ST;  // dummy KiB
      __builtin_amdgcn_raw_ptr_buffer_load_lds(urs, (lds_void*)dst, 16, o, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned o = (kc * kBKd + bk4[i] < K) ? boff[i] + (unsigned)(kc * kBKd * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(hrs, (lds_void*)(sb + (wave * 4 + i) * 256), 16, o, 0, 0, 0);
    }
  };
  // Fragment addresses: row (g*32 + jl) / (wave*64 + r*32 + jl), slot (2G + hf) ^ ((jl >> 2) & 3).
  const int sw = (jl >> 2) & 3;
  const int aoffG[2] = {jl * kBKd + 4 * ((0 + hf) ^ sw), jl * kBKd + 4 * ((2 + hf) ^ sw)};
  const int boffG[2] = {(wave * 64 + jl) * kBKd + 4 * ((0 + hf) ^ sw),
                        (wave * 64 + jl) * kBKd + 4 * ((2 + hf) ^ sw)};
  float4 fa0[NA], fb0[2], fa1[NA], fb1[2];
  auto frag = [&](int kc, int G, float4 (&fa)[NA], float4 (&fb)[2]) {
    const float* sa = ring + (kc % kStages) * ST;
    const float* sb = sa + STA;
#pragma unroll
    for (int g = 0; g < NA; ++g) fa[g] = *reinterpret_cast<const float4*>(sa + g * 32 * kBKd + aoffG[G]);
#pragma unroll
    for (int r = 0; r < 2; ++r) fb[r] = *reinterpret_cast<const float4*>(sb + r * 32 * kBKd + boffG[G]);
  };
  auto mma = [&](const float4 (&fa)[NA], const float4 (&fb)[2]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < NA; ++g)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa[g], s), get4(fb[r], s), acc[g][r], 0, 0, 0);
  };
  constexpr int NRD = NA + 2;                       // fragment reads per half chunk
  constexpr int NMF = 8 * NA;                       // MFMAs per half chunk

  issue(0);
  if (nk > 1) issue(1);
  if (nk > 1) vm_wait<APW + 4>(); else vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  frag(0, 0, fa0, fb0);
  // The schedule is pinned with sched_group_barrier (the compiler otherwise sinks every fragment
  // read to just before the MFMA that consumes it and bunches the DMA issues): each LDS read and
  // each LDS-DMA piece gets an MFMA of its own to hide behind.  The DMA of chunk kc+2 is issued
  // unconditionally (past the last chunk its offsets are out of range: no traffic, zeros into a
  // stage nobody reads), so the loop body is one basic block.
  for (int kc = 0; kc < nk - 1; ++kc) {
    frag(kc, 1, fa1, fb1);
    mma(fa0, fb0);
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NRD, 0);
    __builtin_amdgcn_sched_barrier(0);
    vm_wait<0>();  // this wave's pieces of chunk kc+1 (chunk kc+2 is not issued yet)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue(kc + 2);
    frag(kc + 1, 0, fa0, fb0);
    mma(fa1, fb1);
#pragma unroll
    for (int i = 0; i < APW + 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA piece)
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NRD - APW - 4, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  frag(nk - 1, 1, fa1, fb1);  // last chunk, peeled
  before_last();
  __builtin_amdgcn_sched_barrier(0);
  mma(fa0, fb0);
  mma(fa1, fb1);
}

// LDS floats of mainloop_dma<.., NA>'s ring (3 stages + the dummy-piece KiB when NA is odd).
template <int NA>
constexpr int dma_ring_floats() { return kStages * (NA * 32 * kBKd + kStageB) + ((NA * 2) % 4 ? 256 : 0); }

template <int S>
struct Stage { static constexpr int value = S; };

// mainloop_dma<true, NA> for K % 16 == 0 with no VALU work in the loop: same products, same
// accumulation order, so bitwise the same result.  On gfx950 the fp32 MFMA runs on the VALU
// datapath (tools/mfma_valu_probe.hip: a VALU instruction beside v_mfma_f32_32x32x2_f32 is never
// hidden, ~5 cycles each), so the generic loop's 18 VALU per chunk (DMA offsets with per-lane
// tail checks, stage-relative fragment addresses) cost ~2.4 % of the MFMA time.  Here
//   * every DMA piece keeps a loop-invariant per-lane voffset; the chunk's position goes into the
//     scalar soffset and the LDS stage into M0 (SALU only).  K % 16 == 0 and K <= ldb mean no k
//     tail; rows past nb_valid still read zero from the descriptor's range check; chunks past the
//     end are issued through an empty descriptor (num_records 0: zeros, no traffic);
//   * the loop is unrolled by the 3 ring stages, so every fragment address is a loop-invariant
//     lane base + an immediate offset (ring <= 72 KiB: the 16-bit ds_read offset reaches it).
template <int NA, class BeforeLast>
IADMM_DEV void mainloop_dma_k16(const float* __restrict__ Abase, const float* __restrict__ Bbase, int64_t nb_valid,
                                int ldb, int K, float* ring, floatx16 (&acc)[NA][2], int tid, int wave, int jl,
                                int hf, BeforeLast&& before_last) {
  static_assert(NA == 4 || NA == 5, "A tile = 4 or 5 blocks of 32 rows");
  constexpr int AROWS = NA * 32;
  constexpr int STA = AROWS * kBKd;
  constexpr int ST = STA + kStageB;
  constexpr int NPA = NA * 2;
  constexpr int APW = (NPA + 3) / 4;
  // acc is not zeroed with moves: chunk 0's first MFMA of each accumulator takes an inline-zero C
  // operand instead (128/160 fewer VALU writes per tile; chunk 0 is peeled for that).  At NA = 5
  // the peeled head copies spill a few fragment registers (scratch, outside the loop: the loop
  // itself stays spill- and VALU-free).

  const int lane = tid & 63;
  const int nk = K / kBKd;
  const int nkc32 = (K + kBK - 1) / kBK;
  const int64_t nbv = nb_valid < 256 ? nb_valid : 256;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(Bbase), 0, (int)(nbv * ldb * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(Abase), 0, nkc32 * AROWS * kBK * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Abase), 0, 0, 0x00020000);

  const int prow = lane >> 2, pslot = lane & 3;
  unsigned aoff[APW], boff[4];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int row = (wave + 4 * i) * 16 + prow;
    aoff[i] = (unsigned)(row * kBK + 4 * (pslot ^ ((row >> 2) & 3))) * 4u;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 16 + prow;
    boff[i] = (unsigned)(row * ldb + 4 * (pslot ^ ((row >> 2) & 3))) * 4u;
  }
  auto issue = [&](int kc, auto S) {
    constexpr int s = decltype(S)::value;
    const bool live = kc < nk;
    const __amdgpu_buffer_rsrc_t ua = live ? urs : zrs, hb = live ? hrs : zrs;
    const int sa_off = ((kc >> 1) * AROWS * kBK + (kc & 1) * kBKd) * 4;
    const int sb_off = kc * kBKd * 4;
    float* sa = ring + s * ST;
    float* sb = sa + STA;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int p = wave + 4 * i;
      const bool real = NPA % 4 == 0 || p < NPA;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(real ? ua : zrs, (lds_void*)(real ? sa + p * 256 : ring + kStages * ST),
                                               16, aoff[i], sa_off, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(hb, (lds_void*)(sb + (wave * 4 + i) * 256), 16, boff[i], sb_off, 0, 0);
  };
  const int sw = (jl >> 2) & 3;
  // lane offsets of the fragment reads; laundered through an empty asm once per chunk so the
  // compiler cannot hoist (lane offset + stage/gate constant) sums out of the loop as separate
  // registers: each read stays "lane offset + immediate"
  // LDS byte addresses (ring base folded in) of the fragment reads
  typedef __attribute__((address_space(3))) float lds_float;
  const unsigned rb = (unsigned)(uintptr_t)(lds_float*)ring;
  unsigned aoffG[2] = {rb + (jl * kBKd + 4 * ((0 + hf) ^ sw)) * 4u, rb + (jl * kBKd + 4 * ((2 + hf) ^ sw)) * 4u};
  unsigned boffG[2] = {rb + (STA + (wave * 64 + jl) * kBKd + 4 * ((0 + hf) ^ sw)) * 4u,
                       rb + (STA + (wave * 64 + jl) * kBKd + 4 * ((2 + hf) ^ sw)) * 4u};
  auto launder = [&] {
    asm volatile("" : "+v"(aoffG[0]), "+v"(aoffG[1]), "+v"(boffG[0]), "+v"(boffG[1]));
  };
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const f4v lds_f4;
  auto ld = [](unsigned addr) -> float4 {
    const f4v v = *(lds_f4*)(uintptr_t)addr;
    return make_float4(v.x, v.y, v.z, v.w);
  };
  float4 fa0[NA], fb0[2], fa1[NA], fb1[2];
  auto frag = [&](auto S, int G, float4 (&fa)[NA], float4 (&fb)[2]) {
    constexpr unsigned so = decltype(S)::value * ST * 4u;
#pragma unroll
    for (int g = 0; g < NA; ++g) fa[g] = ld(aoffG[G] + so + g * 32 * kBKd * 4u);
#pragma unroll
    for (int r = 0; r < 2; ++r) fb[r] = ld(boffG[G] + so + r * 32 * kBKd * 4u);
  };
  auto mma = [&](const float4 (&fa)[NA], const float4 (&fb)[2], auto First) {
    constexpr bool first = decltype(First)::value;
    const floatx16 zero = {};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < NA; ++g)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa[g], s), get4(fb[r], s),
                                                           (first && s == 0) ? zero : acc[g][r], 0, 0, 0);
  };
  using No = std::integral_constant<bool, false>;
  using Yes = std::integral_constant<bool, true>;
  constexpr int NRD = NA + 2;
  constexpr int NMF = 8 * NA;
  // one chunk kc (stage S = kc % 3): the schedule of mainloop_dma's loop body
  auto step = [&](int kc, auto S, auto First) {
    constexpr int s = decltype(S)::value;
    launder();
    frag(S, 1, fa1, fb1);
    mma(fa0, fb0, First);
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NRD, 0);
    __builtin_amdgcn_sched_barrier(0);
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue(kc + 2, Stage<(s + 2) % 3>{});
    frag(Stage<(s + 1) % 3>{}, 0, fa0, fb0);
    mma(fa1, fb1, No{});
#pragma unroll
    for (int i = 0; i < APW + 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NRD - APW - 4, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto last = [&](auto S, auto First) {
    frag(S, 1, fa1, fb1);
    before_last();
    __builtin_amdgcn_sched_barrier(0);
    mma(fa0, fb0, First);
    mma(fa1, fb1, No{});
    __builtin_amdgcn_sched_barrier(0);  // nothing of the caller's epilogue moves above these MFMAs
  };

  // Stage numbering is rotated so the peeled last chunk always lands in stage 0 (one copy of the
  // epilogue-operand prefetch): chunk kc uses stage (kc + d) % 3; the r = (nk - 1) % 3 head chunks
  // run before the 3-way unrolled loop.
  const int r = (nk - 1) % 3;
  const int d = (3 - r) % 3;
  if (d == 0) { issue(0, Stage<0>{}); issue(1, Stage<1>{}); }  // chunk 1 past the end when nk == 1:
  else if (d == 1) { issue(0, Stage<1>{}); issue(1, Stage<2>{}); }  // zeros into a stage nobody reads
  else { issue(0, Stage<2>{}); issue(1, Stage<0>{}); }
  vm_wait<APW + 4>();
  __builtin_amdgcn_s_barrier();
  if (d == 0) frag(Stage<0>{}, 0, fa0, fb0);
  else if (d == 1) frag(Stage<1>{}, 0, fa0, fb0);
  else frag(Stage<2>{}, 0, fa0, fb0);
  int kc;
  if (nk == 1) {
    last(Stage<0>{}, Yes{});
    return;
  }
  if (r == 2) {
    step(0, Stage<1>{}, Yes{});
    step(1, Stage<2>{}, No{});
    kc = 2;
  } else if (r == 1) {
    step(0, Stage<2>{}, Yes{});
    kc = 1;
  } else {  // nk - 1 = 3, 6, ...
    step(0, Stage<0>{}, Yes{});
    step(1, Stage<1>{}, No{});
    step(2, Stage<2>{}, No{});
    kc = 3;
  }
  for (; kc < nk - 1; kc += 3) {
    step(kc, Stage<0>{}, No{});
    step(kc + 1, Stage<1>{}, No{});
    step(kc + 2, Stage<2>{}, No{});
  }
  last(Stage<0>{}, No{});
}

// The cell's instance: A = the packed gate weights of hidden tile jt, B = the H panel of rows
// [rbase, rbase + 256).  K16: h % 16 == 0 (mainloop_dma_k16).
template <bool K16, class BeforeLast>
IADMM_DEV void cell_mainloop_dma(const float* __restrict__ H, int64_t M, int h, int nkc32,
                                 const float* __restrict__ Ubase, int64_t rbase, float* ring,
                                 floatx16 (&acc)[4][2], int tid, int wave, int jl, int hf,
                                 BeforeLast&& before_last) {
  (void)nkc32;
  if constexpr (K16)
    mainloop_dma_k16<4>(Ubase, H + rbase * h, M - rbase, h, h, ring, acc, tid, wave, jl, hf, before_last);
  else
    mainloop_dma<true>(Ubase, 128, kBK, H + rbase * h, M - rbase, h, h, ring, acc, tid, wave, jl, hf,
                       before_last);
}

// The fused cell epilogue: gates, C' = I U + F C, H' = O tanh(C'), projection partial, from the
// accumulators of a 32-unit x (wave's 64 rows) tile.
// Split in two so a kernel can issue the global loads (cell_epi_load) early, e.g. before its last
// K chunk, and keep them in registers until cell_epi_compute.
// accumulator element q of lane (jl,hf): hidden jj = (q&3) + 8*(q>>2) + 4*hf, data row jl.
struct CellEpiIn {
  float4 cold[2][4];  // C[R, jt*32 + 8*qq + 4*hf .. +4] for the lane's two rows
  float in0[2], in1[2];
};

template <bool VEC>
IADMM_DEV void cell_epi_load(const CellArgsT& a, int jt, int64_t rbase, int wave, int jl, int hf, CellEpiIn& e) {
  const int h = a.h;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = rbase + wave * 64 + r * 32 + jl;
    const bool rok = R < a.M;
    e.in0[r] = rok ? a.xv[R] : 0.f;
    e.in1[r] = rok ? a.g[R] : 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int j0 = jt * kJT + 8 * qq + 4 * hf;
      if constexpr (VEC) {
        e.cold[r][qq] = (rok && j0 < h) ? *reinterpret_cast<const float4*>(a.C + R * h + j0)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) set4(e.cold[r][qq], k, (rok && j0 + k < h) ? a.C[R * h + j0 + k] : 0.f);
      }
    }
  }
}

// Packed epilogue: unit pairs (jj, jj+1) go through v_pk_*_f32 together (common.h *_cell2).
// sWp = the tile's Wx fields as [16 unit pairs][16 fields][2 units] (cell_fill_wpairs), so one
// float4 holds two fields of both units of a pair.  The projection partial runs as two interleaved
// sums (even / odd unit of each pair) added at the end.
IADMM_DEV void cell_fill_wpairs(const float* __restrict__ Wx, int jt, float* sWp, int tid, int nthreads) {
  for (int i = tid; i < kWxF * kJT; i += nthreads) {
    const int pr = i >> 5, f = (i >> 1) & 15, u = i & 1;
    sWp[i] = Wx[(int64_t)(jt * kJT + 2 * pr + u) * kWxF + f];
  }
}

template <bool VEC, int DIAG = 0>
IADMM_DEV void cell_epi_compute(const CellArgsT& a, floatx16 (&acc)[4][2], const float* sWp, int jt,
                                int64_t rbase, int wave, int jl, int hf, const CellEpiIn& ei) {
  const int h = a.h;
  const int64_t M = a.M;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = rbase + wave * 64 + r * 32 + jl;
    const bool rok = R < M;
    const float2v in0 = splat2(ei.in0[r]), in1 = splat2(ei.in1[r]);
    float2v gs = splat2(0.f);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      __builtin_amdgcn_sched_barrier(0);  // one (rows, 4 units) group at a time: bounded live range
      const int jj0 = 8 * qq + 4 * hf;
      const int j0 = jt * kJT + jj0;
      const float4 cold = ei.cold[r][qq];
      float4 cnew, hnew;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        // fields 0..13 of units (jj0 + 2pp, +1): 7 float4 of one 128-B sWp row (broadcast across
        // the 32 lanes of a half-wave)
        const float4* wp = reinterpret_cast<const float4*>(sWp + ((jj0 >> 1) + pp) * 32);
        float4 w4[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) w4[i] = wp[i];
        auto fld = [&](int f) -> float2v {
          const float4& t = w4[f >> 1];
          return (f & 1) ? float2v{t.z, t.w} : float2v{t.x, t.y};
        };
        const int q = qq * 4 + 2 * pp;
        float2v pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pre[g] = cell_pre2(in0, in1, float2v{acc[g][r][q], acc[g][r][q + 1]}, fld(3 * g), fld(3 * g + 1),
                             fld(3 * g + 2));
        }
        const float2v ig = sigmoid_cell2(pre[0]), fg = sigmoid_cell2(pre[1]), og = sigmoid_cell2(pre[2]);
        const float2v ug = tanh_cell2(pre[3]);
        const float2v cv = pp ? float2v{cold.z, cold.w} : float2v{cold.x, cold.y};
        const float2v c2 = ig * ug + fg * cv;
        const float2v h2 = og * tanh_cell2(c2);
        gs = fma2(h2, fld(12), gs);
        if (pp == 0) { cnew.x = c2.x; cnew.y = c2.y; hnew.x = h2.x; hnew.y = h2.y; }
        else         { cnew.z = c2.x; cnew.w = c2.y; hnew.z = h2.x; hnew.w = h2.y; }
      }
      if (DIAG == 2) {  // timing diagnostic: no H'/C' stores (keep the values alive)
        gs.x += cnew.x + cnew.y + cnew.z + cnew.w;
      } else if (rok) {
        if constexpr (VEC) {
          if (j0 < h) {
            *reinterpret_cast<float4*>(a.Cn + R * h + j0) = cnew;
            *reinterpret_cast<float4*>(a.Hn + R * h + j0) = hnew;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (j0 + e < h) {
              a.Cn[R * h + j0 + e] = get4(cnew, e);
              a.Hn[R * h + j0 + e] = get4(hnew, e);
            }
          }
        }
      }
    }
    float gsum = gs.x + gs.y;
    gsum += __shfl_xor(gsum, 32, 64);
    if (hf == 0 && rok) a.part[(int64_t)jt * M + R] = gsum;
  }
}

// The DMA kernel's epilogue on buffer loads/stores (h % 4 == 0).  Every global access of the
// epilogue goes through a descriptor based at the workgroup's row panel whose range ends at its last
// valid row: rows past M read 0 / are dropped by the range check (no exec-mask branches, no
// zeroing moves), and each lane needs one 32-bit offset per row block, the unit groups (qq) being
// immediate offsets -- a fraction of the 64-bit address VALU of cell_epi_load / cell_epi_compute.
// (Each VALU instruction here costs the SIMD's fp32-MFMA stream its issue cycles:
// tools/mfma_valu_probe.hip.)  Same arithmetic as cell_epi_compute: bitwise the same results.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
struct CellEpiBuf {
  __amdgpu_buffer_rsrc_t c, cn, hn, xv, g, part;
  unsigned vo[2];    // bytes: (row block r of the lane, units jt*32 + 4*hf) inside the panel
  unsigned vr[2];    // bytes: row of the lane inside the panel (xv, g); part: out of range for hf = 1
  unsigned qadd[4];  // tail hidden tile only: qq*32 B, or out of range past h
  bool full;         // the hidden tile has all 32 units (uniform)
  float4 cold[2][4];
  float in0[2], in1[2];
};

IADMM_DEV void cell_epi_setup_buf(const CellArgsT& a, int jt, int64_t rbase, int wave, int jl, int hf, CellEpiBuf& e) {
  const int h = a.h;
  const int64_t M = a.M;
  const int nvalid = (int)((M - rbase) < kRows ? (M - rbase) : kRows);
  const int64_t pan = rbase * h;
  e.c = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.C + pan), 0, nvalid * h * 4, 0x00020000);
  e.cn = __builtin_amdgcn_make_buffer_rsrc(a.Cn + pan, 0, nvalid * h * 4, 0x00020000);
  e.hn = __builtin_amdgcn_make_buffer_rsrc(a.Hn + pan, 0, nvalid * h * 4, 0x00020000);
  e.xv = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xv + rbase), 0, nvalid * 4, 0x00020000);
  e.g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.g + rbase), 0, nvalid * 4, 0x00020000);
  e.part = __builtin_amdgcn_make_buffer_rsrc(a.part + (int64_t)jt * M + rbase, 0, nvalid * 4, 0x00020000);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const unsigned row = (unsigned)(wave * 64 + r * 32 + jl);
    e.vo[r] = (row * (unsigned)h + (unsigned)(jt * kJT + 4 * hf)) * 4u;
    e.vr[r] = row * 4u;
  }
  e.full = (jt + 1) * kJT <= h;
  if (!e.full) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) e.qadd[qq] = jt * kJT + 8 * qq + 4 * hf < h ? 32u * qq : 0x80000000u;
  }
}

IADMM_DEV float4 u2f4(u32x4 v) {
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
IADMM_DEV u32x4 f42u(float4 v) {
  return u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
}

IADMM_DEV void cell_epi_load_buf(CellEpiBuf& e) {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    e.in0[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(e.xv, e.vr[r], 0, 0));
    e.in1[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(e.g, e.vr[r], 0, 0));
    if (e.full) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) e.cold[r][qq] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(e.c, e.vo[r] + 32u * qq, 0, 0));
    } else {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) e.cold[r][qq] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(e.c, e.vo[r] + e.qadd[qq], 0, 0));
    }
  }
}

template <int DIAG = 0>
IADMM_DEV void cell_epi_compute_buf(floatx16 (&acc)[4][2], const float* sWp, int hf, CellEpiBuf& e) {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float2v gs = splat2(0.f);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      __builtin_amdgcn_sched_barrier(0);  // one (rows, 4 units) group at a time: bounded live range
      const int jj0 = 8 * qq + 4 * hf;
      const float4 cold = e.cold[r][qq];
      // both unit pairs of the group at once (float4v: two independent packed halves)
      const float4* wp0 = reinterpret_cast<const float4*>(sWp + (jj0 >> 1) * 32);
      const float4* wp1 = wp0 + 8;  // next pair's 128-B row
      float4 w0[7], w1[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) { w0[i] = wp0[i]; w1[i] = wp1[i]; }
      auto fld4 = [&](int f) -> float4v {
        const float4& t0 = w0[f >> 1];
        const float4& t1 = w1[f >> 1];
        return (f & 1) ? float4v{t0.z, t0.w, t1.z, t1.w} : float4v{t0.x, t0.y, t1.x, t1.y};
      };
      const int q = qq * 4;
      const float4v in0v = splat4(e.in0[r]), in1v = splat4(e.in1[r]);
      float4v pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        pre[g] = cell_pre4(in0v, in1v, float4v{acc[g][r][q], acc[g][r][q + 1], acc[g][r][q + 2], acc[g][r][q + 3]},
                           fld4(3 * g), fld4(3 * g + 1), fld4(3 * g + 2));
      const float4v ig = sigmoid_cell4(pre[0]), fg = sigmoid_cell4(pre[1]), og = sigmoid_cell4(pre[2]);
      const float4v ug = tanh_cell4(pre[3]);
      const float4v cv = float4v{cold.x, cold.y, cold.z, cold.w};
      const float4v c4 = ig * ug + fg * cv;
      const float4v h4 = og * tanh_cell4(c4);
      const float4v wh = fld4(12);
      gs = fma2(float2v{h4.x, h4.y}, float2v{wh.x, wh.y}, gs);
      gs = fma2(float2v{h4.z, h4.w}, float2v{wh.z, wh.w}, gs);
      const float4 cnew = make_float4(c4.x, c4.y, c4.z, c4.w), hnew = make_float4(h4.x, h4.y, h4.z, h4.w);
      if (DIAG == 2) {  // timing diagnostic: no H'/C' stores (keep the values alive)
        gs.x += cnew.x + cnew.y + cnew.z + cnew.w;
      } else {
        const unsigned o = e.vo[r] + (e.full ? 32u * qq : e.qadd[qq]);
        __builtin_amdgcn_raw_buffer_store_b128(f42u(cnew), e.cn, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(f42u(hnew), e.hn, o, 0, 0);
      }
    }
    float gsum = gs.x + gs.y;
    gsum += __shfl_xor(gsum, 32, 64);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gsum), e.part, hf ? 0x80000000u : e.vr[r], 0, 0);
  }
}

template <bool VEC>
IADMM_DEV void cell_epilogue(const CellArgsT& a, floatx16 (&acc)[4][2], const float* sW, int jt,
                             int64_t rbase, int wave, int jl, int hf) {
  CellEpiIn ei;
  cell_epi_load<VEC>(a, jt, rbase, wave, jl, hf, ei);
  cell_epi_compute<VEC>(a, acc, sW, jt, rbase, wave, jl, hf, ei);
}

// The forward cell kernel (production instance: NW = 4, PRIO = 0, lstm.hip): fp32-MFMA gate GEMM
// (cell_mainloop) + the fused cell epilogue.  Workgroup = 32 hidden units x 64*NW rows.
template <bool VEC, int NW = 4, int PRIO = 0, bool BUF = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void cell_fwd_kernel(CellArgsT a) {
  constexpr int ROWS = 64 * NW;
  __shared__ __attribute__((aligned(16))) float sA[128 * kLD];
  __shared__ __attribute__((aligned(16))) float sB[ROWS * kLD];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];

  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jl = lane & 31, hf = lane >> 5;
  const int h = a.h;
  const int64_t M = a.M;
  const int64_t rbase = (int64_t)rt * ROWS;

  cell_fill_wpairs(a.Wx, jt, sW, tid, 64 * NW);

  floatx16 acc[4][2];
  cell_mainloop<VEC, NW, PRIO, BUF>(a.H, M, h, a.nkc32, a.Upk + (int64_t)jt * a.nkc32 * 128 * kBK, rbase, sA, sB,
                               acc, tid, wave, jl, hf);

  cell_epilogue<VEC>(a, acc, sW, jt, rbase, wave, jl, hf);
}


// Forward cell kernel on the LDS-DMA main loop (VEC only: h % 4 == 0, 16-B aligned rows); K16:
// h % 16 == 0, the VALU-free loop (mainloop_dma_k16).
// Dynamic LDS: kRingFloats + kWxF*kJT floats (74 KiB) -> 2 workgroups per CU.
// DIAG (timing tools only): 1 = skip the epilogue (main-loop cost); 2 = epilogue without the
// H'/C' stores; 3 = epilogue without the C / xv / g loads.
// DIAG 4: as 0, plus s_memtime stamps (kernel start, main loop end, epilogue operands landed,
// epilogue end) of wave 0 of every workgroup into a.part[njt * M ...]; 5: same without the H'/C'
// stores; 6: as 4 plus HW_ID / XCC_ID (8 words per workgroup: co-residency phase study) --
// diagnostic builds only (tools/cellbench).
template <int DIAG = 0, bool K16 = false>
__global__ __launch_bounds__(256, 2) void cell_fwd_dma_kernel(CellArgsT a) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  uint64_t t_start = 0, t_ml = 0;
  if constexpr (DIAG == 4 || DIAG == 6) t_start = __builtin_amdgcn_s_memtime();
  float* ring = dsm;
  float* sW = dsm + kRingFloats;
  int jt, rt;
  cell_tile_of_block_grouped(a.njt, (a.M + kRows - 1) / kRows, a.pgroup, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int jl = lane & 31, hf = lane >> 5;
  const int64_t rbase = (int64_t)rt * kRows;
  cell_fill_wpairs(a.Wx, jt, sW, tid, 256);
  // sW visible to every wave.  Here rather than after the main loop: a fence there would wait
  // (vmcnt) for the epilogue operands prefetched behind the last chunk, and the compiler may sink
  // the last chunk's MFMAs below the barrier, exposing that load latency.
  __syncthreads();
  floatx16 acc[4][2];
  CellEpiBuf ei;
  cell_epi_setup_buf(a, jt, rbase, wave, jl, hf, ei);
  cell_mainloop_dma<K16>(a.H, a.M, a.h, a.nkc32, a.Upk + (int64_t)jt * a.nkc32 * 128 * kBK, rbase, ring, acc,
                    tid, wave, jl, hf, [&] {
                      if constexpr (DIAG == 3) {
#pragma unroll
                        for (int r = 0; r < 2; ++r) {
                          ei.in0[r] = ei.in1[r] = 0.5f;
#pragma unroll
                          for (int qq = 0; qq < 4; ++qq) ei.cold[r][qq] = make_float4(0.1f, 0.2f, 0.3f, 0.4f);
                        }
                      } else {
                        cell_epi_load_buf(ei);
                      }
                    });
  if constexpr (DIAG == 1) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q) t += acc[g][r][q];
    a.part[(int64_t)blockIdx.x * 256 + tid] = t;
    return;
  }
  uint64_t t_c = 0;
  if constexpr (DIAG >= 4) {
    t_ml = __builtin_amdgcn_s_memtime();
    vm_wait<0>();  // the prefetched epilogue operands
    t_c = __builtin_amdgcn_s_memtime();
  }
  cell_epi_compute_buf<(DIAG == 4 || DIAG == 6) ? 0 : (DIAG == 5 ? 2 : DIAG)>(acc, sW, hf, ei);
  if constexpr (DIAG >= 4) {
    const uint64_t t_end = __builtin_amdgcn_s_memtime();
    if (tid == 0) {
      constexpr int W = DIAG == 6 ? 8 : 4;
      uint64_t* st = reinterpret_cast<uint64_t*>(a.part + (int64_t)a.njt * a.M) + (int64_t)blockIdx.x * W;
      st[0] = t_start; st[1] = t_ml; st[2] = t_c; st[3] = t_end;
      if constexpr (DIAG == 6) {
        st[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        st[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
      }
    }
  }
}
constexpr int kDmaLdsBytes = (kRingFloats + kWxF * kJT) * 4;

}  // namespace iadmm
