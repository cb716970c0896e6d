// Implicit-GEMM convolutions on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Replaces torch.nn.Conv2d / ConvTranspose2d forward and aten::convolution_backward
// on the reference's hot path (GLI:336,361,387,410,428,448; arch 1 GLI:202-223,260-302).
//
// Three GEMM modes, one kernel template:
//   MODE_CONV   C[m][n] = sum_k im2col(x)[m][k] * Wp[k][n]       (Conv2d fwd, ConvT dgrad,
//               stride-1 ConvT fwd / Conv dgrad with a flipped kernel, 1x1 "GEMM" layers)
//   MODE_CONVT2 the same per output phase (oh%2, ow%2) of a k4 s2 p1 ConvTranspose2d
//               (ConvT fwd, Conv dgrad): 4 sub-pixel GEMMs with K = 4*Cin, no zero taps
//   MODE_WGRAD  C[m][n] = sum_p G[p][m] * im2col(img)[p][n]       (weight gradients)
// Activations are NHWC (torch channels_last) inside the path; any (b,c,h,w) strides are
// accepted (NCHW images at the boundary take the scalar gather).  fp32 in, fp32 MFMA
// accumulate: no reduced precision anywhere.
//
// Tiling: 256 threads = 4 waves; block tile BM x BN x BK(32); each wave owns a
// (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA accumulators.  LDS is double buffered with
// register-staged global loads (next tile's loads in flight while the current tile's
// MFMAs run).  LDS images keep every MFMA operand read a conflict-free ds_read_b32:
// m-major tiles use row stride BK+1, k-major tiles BM+4 / BN+4.  Split-K writes fp32
// slabs reduced in fixed order (deterministic) by splitk_reduce.
#include "common.h"

#include <string>
#include <type_traits>
#include <atomic>
#include <vector>

namespace rgan {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Raw-buffer byte offset past every record of a descriptor (< 2^31 bytes): loads return 0.
constexpr int OOB = (int)0x80000000;
// fast-path tensors must fit a buffer descriptor with this margin
constexpr long long FAST_MAX_BYTES = (1LL << 31) - (1LL << 24);

enum { MODE_CONV = 0, MODE_CONVT2 = 1, MODE_WGRAD = 2, MODE_NARROW_T = 3, MODE_NARROW_IN = 4, MODE_DENSE1 = 5,
       MODE_NARROW3 = 6, MODE_NARROW3W = 7 };
constexpr int BK = 32;
// split-K occupancy target (blocks): two resident 256-thread blocks per CU on 256 CUs
constexpr long long SPLIT_TARGET = 512;

// n / d for 0 <= n < 2^31 via multiply-high (host-computed magic numbers)
struct FastDiv {
  uint32_t d, m, l;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) {
    d = div;
    l = 0;
    while ((1u << l) < d) ++l;
    uint64_t one = 1;
    m = (uint32_t)(((one << 32) * ((one << l) - d)) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    uint32_t hi = __umulhi(n, m);
    return (uint32_t)(((uint64_t)hi + n) >> l);
  }
};

struct Img {
  const float* p;
  long long sb, sc, sh, sw;
  int H, W, C;
};

struct OutMap {
  FastDiv fgw, fghw;      // row m -> (b, i, j) over (gh, gw)
  int step;
  long long sb, sh, sw;
  FastDiv fnc, fnkw;      // col n -> (nh, nw, c) over (nkh, nkw, nc)
  long long th, tw, tc;
};

struct GemmArgs {
  int M, N, K;
  int ksplit, splits, tiles_n;
  Img a;                  // CONV/CONVT2: x.  WGRAD: gradient image (channel = m)
  Img im;                 // WGRAD: image expanded by im2col
  int KH, KW, stride, pad;
  FastDiv fgw, fghw;      // decomposition of m (CONV/CONVT2) or p (WGRAD)
  FastDiv fC, fKW;        // k (CONV/CONVT2) or n (WGRAD) -> (kh, kw, ci)
  const float* Bw;        // packed weights [phase][N][K]
  float* C;
  OutMap out;
  const float* bias;
  const float* wscale;    // nullable device scalar multiplying the accumulator (spectral 1/sigma)
  int act;
  float alpha;
  float* slab;
  // FAST paths (raw buffer loads, scalar per-tile offsets): descriptor sizes in bytes
  int a_bytes, im_bytes, bw_bytes;
  int im_buf;             // non-FAST WGRAD: the scalar im2col gathers through the im_bytes descriptor
  int vec_out;            // output n-quads contiguous and 16-B aligned (host-checked)
  int xgroup, nph;        // tile order (0: default; 2: blocks sharing weight columns on one XCD; 3: band order,
                          // each XCD a contiguous eighth of the m tiles); phases
  double* bnp;            // nullable: BatchNorm moments of every 64-row output segment (vector epilogue)
  int accum;              // WGRAD: add into C (gradient accumulation) instead of overwriting it
  // FAST conv WGRAD with a bias (rgan_conv_wgrad dbias): the bias gradient sum_p dy[p][m] is
  // formed from the A tiles the GEMM stages anyway (the n-tile-0 blocks); unsplit: written to
  // dbias (added when db_accum), split: per-split doubles dbp[split][M], summed in split order
  // by the WGRAD reduce
  double* dbp;
  float* dbias;
  int db_accum;
  int db_k0;              // first pixel row summed into dbias (a multiple of BK; rgan_conv_wgrad_rows)
  // Post-op for the layer that PRODUCED this GEMM's output operand (rgan_conv_post: a data
  // gradient, or G's image-layer gradient GEMM), applied where the value is final (unsplit
  // epilogue or split-K reduce); px has C's layout (host-checked):
  //   pmode 1: C = v * act'(px), px = the producer's activation output (its act backward);
  //   pmode 2: C = g = v * act'(px * al + be), px = the producer's BatchNorm input y, al/be
  //            from (mean, invstd) pst[k][2N] of batch segment k and gamma/beta, plus the
  //            BatchNorm backward sums (sum g, sum g (y - mean)) of every 64-row segment into
  //            ppart[seg][2][N] in double (seg as bnp's) -- the bn_bwd_partial pass.
  const float* px;
  const float* pst;
  const float* pgam;
  const float* pbet;
  double* ppart;
  int pmode, pact, pnseg;
  float palpha;
};

// per-channel BatchNorm affine of the producer (pmode 2): z = y * al + be
__device__ __forceinline__ void post_consts(const GemmArgs& g, int k, int n, float& al, float& be, float& mu) {
  const int c = min(n, g.N - 1);
  const float* st = g.pst + (size_t)k * 2 * g.N;
  mu = st[c];
  al = (g.pgam ? g.pgam[c] : 1.f) * st[g.N + c];
  be = (g.pbet ? g.pbet[c] : 0.f) - mu * al;
}

// batch segment of output row m (pmode 2, pnseg equal segments of the M rows of every phase)
__device__ __forceinline__ int post_seg(const GemmArgs& g, int m) {
  return g.pnseg > 1 ? m / (g.M / g.pnseg) : 0;
}

__device__ __forceinline__ long long row_offset(const OutMap& o, int m, int phase) {
  uint32_t b = o.fghw.div(m);
  uint32_t rem = m - b * o.fghw.d;
  uint32_t i = o.fgw.div(rem);
  uint32_t j = rem - i * o.fgw.d;
  int ph = phase >> 1, pw = phase & 1;
  return (long long)b * o.sb + (long long)(i * o.step + ph) * o.sh + (long long)(j * o.step + pw) * o.sw;
}

__device__ __forceinline__ long long col_offset(const OutMap& o, int n) {
  uint32_t t = o.fnc.div(n);
  uint32_t c = n - t * o.fnc.d;
  uint32_t nh = o.fnkw.div(t);
  uint32_t nw = t - nh * o.fnkw.d;
  return (long long)nh * o.th + (long long)nw * o.tw + (long long)c * o.tc;
}

// FAST (AV && BV only; host checks the conditions in set_fast): every BK tile of a
// CONV/CONVT2 GEMM lies inside one filter tap (Cin % BK == 0), so per-row input offsets
// change only when the tap does and the per-tile advance (channel chunk, weight row
// block) is a wave-uniform scalar passed as the buffer load's soffset: the main loop
// issues almost no VALU (fp32 MFMA shares the VALU datapath on gfx950 --
// SQ_VALU_MFMA_COEXEC_CYCLES = 0 -- so every address instruction costs MFMA cycles).
// WGRAD: the gradient rows are pixel-contiguous (offset = p * pixel stride: scalar
// advance) and the im2col operand reads one tap per block tile (Cin % BN == 0) through
// a per-tile table of pixel offsets built by one wave into LDS two tiles ahead.
template <int MODE, int BM, int BN, int WM, int WN, bool AV, bool BV, bool FAST, bool EMU, bool POST = false>
__device__ __forceinline__ void gemm_body(const GemmArgs& g) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM * WN == 4, "tile config");
  constexpr bool AK = (MODE == MODE_WGRAD);          // A staged k-major
  // KROW (every FAST path): both operands staged as k-contiguous rows ([m][k], [n][k]);
  // every lane reads 4 consecutive k of its row with one conflict-free ds_read_b128 that
  // feeds 4 MFMA steps.  The k order inside a BK tile is permuted (MFMA step s of lane
  // half h takes k = 16h + s), the same for A and B, so only the fp32 summation order
  // changes.  CONV/CONVT2: the global rows are k-contiguous too (channels; [N][K] weight
  // pack), stores are ds_write_b128 and the row stride is 36 dwords (9 slots: 16 rows hit
  // 16 slots).  WGRAD (SWZ): k = pixel is the global outer index, so each float4 (4
  // consecutive m or n of one pixel) is stored transposed as 4 ds_write_b32 into rows of
  // 32 dwords whose 16-B quads are XOR-swizzled by (row >> 1) & 7: the reads stay
  // conflict-free (slot = 8 (row & 1) + quad ^ swz) and each store instruction (8 channel
  // quads x 4 pixels per half-wave) is at most 2-way (free for ds_write_b32).
  constexpr bool KROW = FAST;
  constexpr bool SWZ = FAST && MODE == MODE_WGRAD;
  constexpr int KROW_LD = SWZ ? BK : BK + 4;
  constexpr int A_LD = KROW ? KROW_LD : AK ? (BM + 4) : (BK + 1);
  constexpr int A_SZ = KROW ? BM * KROW_LD : AK ? BK * (BM + 4) : BM * (BK + 1);
  constexpr int B_LD = KROW ? KROW_LD : BN + 4;
  constexpr int B_SZ = KROW ? BN * KROW_LD : BK * B_LD;
  constexpr int STAGE = A_SZ + B_SZ;
  // The 256x32 narrow-N tile (CFG_N) is single-buffered (two barriers per k tile): its two
  // stages (83 KB) left one resident block per CU; one stage (41.5 KB) gives three.  The
  // 128x64 tile (CFG_M) likewise (two -> five blocks; C3h32 -1.6 %, C1 / C4 unchanged).  The
  // 128x128 tile keeps two stages (single-buffered it lost 9 %: its vector epilogue needs the
  // LDS, and two blocks per CU already hide the one barrier).  The 64x64 tile (CFG_S: small
  // forward / data-gradient GEMMs, one 32x32 accumulator per wave) keeps two stages (36 KB)
  constexpr bool GEMM_SB = !EMU && ((BM == 256 && BN == 32) || (BM == 128 && BN == 64));
  constexpr int EPI_SZ = KROW ? 4 * (GEMM_SB ? 32 : 64) * 72 : 0;  // vector epilogue staging (4 waves x rows x 72)
  // EMU: one (single-buffered) stage of six bf16 planes (A hi/mid/lo, B hi/mid/lo), rows of
  // 32 bf16 = 16 dwords at a 20-dword stride (16 lanes' ds_read_b128 on 16 distinct quads)
  constexpr int EMU_RS = 20, EMU_PLANE = 128 * EMU_RS;  // dwords
  constexpr int MAIN_SZ = EMU ? 6 * EMU_PLANE : GEMM_SB ? STAGE : 2 * STAGE;
  static_assert(!EMU || (FAST && MODE != MODE_WGRAD && BM == 128 && BN == 128), "bf16x6 path: FAST 128x128 CONV/CONVT2");
  __shared__ __attribute__((aligned(16))) float smem[MAIN_SZ > EPI_SZ ? MAIN_SZ : EPI_SZ];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid / WN) * (BM / WM), wn = (wid % WN) * (BN / WN);
  // Tile order.  Default: x = (m tile, n tile), z = (phase, split).  Blocks are dispatched
  // round-robin over the 8 XCDs, so blocks that read the same operand rows are put 8 dispatch
  // slots apart -- one XCD, one L2 -- instead of on 4-8 different L2s.  (The first such
  // order, xgroup 1 -- the n tiles and phases of one m tile on one XCD -- was superseded by
  // the band order 3 below; tools/patches/xgroup1_row_grouping.diff.)  xgroup 2 (layers whose weights outweigh
  // their input: the deep D convs, G's deep data gradients / ConvTs): the blocks that read
  // the same weight columns (the m tiles and phases of one n tile) share an XCD instead, so
  // the weight is fetched into one L2 rather than into every L2 once per m tile.
  int tm_i, tn_i, phase, split, z;
  if (g.xgroup == 2) {
    const int b = blockIdx.x, r = b >> 3, tiles_m = (g.M + BM - 1) / BM, per = tiles_m * g.nph;
    const int q = r % per;
    tn_i = (r / per) * 8 + (b & 7);
    tm_i = q % tiles_m;
    phase = q / tiles_m;
    split = blockIdx.z;
    z = phase * g.splits + split;
  } else if (g.xgroup == 3) {
    // band order: XCD x (dispatch slot b % 8) takes the x-th eighth of the m tiles, in order,
    // each m tile's n tiles and phases back to back -- the blocks in flight on one XCD cover
    // consecutive output rows, which read overlapping input rows (4 x 4 windows, stride 2)
    const int b = blockIdx.x, r = b >> 3, per = g.tiles_n * g.nph;
    const int q = r % per;
    tm_i = (b & 7) * ((g.M + BM - 1) / BM / 8) + r / per;
    tn_i = q % g.tiles_n;
    phase = q / g.tiles_n;
    split = blockIdx.z;
    z = phase * g.splits + split;
  } else {
    const int tile = blockIdx.x;
    tm_i = tile / g.tiles_n;
    tn_i = tile - tm_i * g.tiles_n;
    z = blockIdx.z;
    phase = z / g.splits;
    split = z - phase * g.splits;
  }
  const int m0 = tm_i * BM, n0 = tn_i * BN;
  const int kbeg = split * g.ksplit;
  const int kend = min(g.K, kbeg + g.ksplit);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int ph = phase >> 1, pw = phase & 1;
  const float* __restrict__ Bw = g.Bw + (size_t)phase * g.K * g.N;

  // ---------------- per-thread load geometry ----------------
  // A (CONV/CONVT2, vector): rows (tid>>3)+32i, quad tid&7
  constexpr int AR = BM / 32;
  long long abase[(MODE != MODE_WGRAD && AV) ? AR : 1];
  int aih[(MODE != MODE_WGRAD && AV) ? AR : 1], aiw[(MODE != MODE_WGRAD && AV) ? AR : 1];
  if constexpr (MODE != MODE_WGRAD && AV) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int m = m0 + (tid >> 3) + 32 * i;
      if (m < g.M) {
        uint32_t b = g.fghw.div(m);
        uint32_t rem = m - b * g.fghw.d;
        uint32_t oi = g.fgw.div(rem);
        uint32_t oj = rem - oi * g.fgw.d;
        abase[i] = (long long)b * g.a.sb;
        if constexpr (MODE == MODE_CONV) {
          aih[i] = (int)oi * g.stride - g.pad;
          aiw[i] = (int)oj * g.stride - g.pad;
        } else {
          aih[i] = (int)oi;
          aiw[i] = (int)oj;
        }
      } else {
        abase[i] = 0;
        aih[i] = -(1 << 28);
        aiw[i] = 0;
      }
    }
  }
  // WGRAD B (vector): fixed column quad n = n0 + 4*(tid % (BN/4)) -> (kh, kw, ci)
  int wb_kh = 0, wb_kw = 0, wb_ci = 0;
  bool wb_nok = false;
  if constexpr (MODE == MODE_WGRAD && BV) {
    int n = n0 + 4 * (tid % (BN / 4));
    wb_nok = n < g.N;
    uint32_t t = g.fC.div(n);
    wb_ci = n - t * g.fC.d;
    wb_kh = g.fKW.div(t);
    wb_kw = t - wb_kh * g.fKW.d;
  }

  // register staging
  constexpr int A_ELEMS = BM * BK / 256;   // floats per thread
  constexpr int B_ELEMS = BK * BN / 256;
  float ra[A_ELEMS];
  float rb[B_ELEMS];

  // ---------------- FAST-path state ----------------
  static_assert(!FAST || (AV && BV), "FAST needs vector operands");
  // WGRAD FAST thread map (per operand of R rows = BM or BN): tid -> quad q = (tid&7) +
  // 8 ((tid>>5) % (R/32)), pixels p = ((tid>>3)&3) + 4 ((tid>>5) / (R/32)) + (32/(R/32)) i
  constexpr int FA_N = (MODE == MODE_WGRAD) ? BM / 32 : AR;  // A loads per thread
  constexpr int FB_N = BN / 32;
  auto sw_q = [&](int R) { return (tid & 7) + 8 * ((tid >> 5) % (R / 32)); };
  auto sw_p = [&](int R, int i) { return ((tid >> 3) & 3) + 4 * ((tid >> 5) / (R / 32)) + (32 / (R / 32)) * i; };
  // WGRAD FAST: im2col pixel offsets of the next tiles, per tap of the block's n tile (a
  // tile holds one tap when Cin >= BN, else BN / Cin <= 4 whole taps of one kernel row)
  __shared__ int ptab[2][4 * BK];
  __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g.a.p, (short)0, g.a_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t brsrc =
      MODE == MODE_WGRAD ? __builtin_amdgcn_make_buffer_rsrc((void*)g.im.p, (short)0, g.im_bytes, 0x00020000)
                         : __builtin_amdgcn_make_buffer_rsrc((void*)Bw, (short)0, g.bw_bytes, 0x00020000);
  int aoff[FAST ? FA_N : 1], boff[FAST ? FB_N : 1];
  int f_tap = 0, f_c0 = 0, f_cin = 1, w_tab = 0;
  int w_ntap = 1, w_tq = 0, w_qb = 0;  // WGRAD FAST: taps per n tile; this thread's tap, channel byte offset
  int st_k0 = 0;                        // WGRAD FAST: first pixel row of the tile in the staging registers
  if constexpr (FAST) {
    if constexpr (MODE != MODE_WGRAD) {
      // packed weights [N][K]: rows n = n0 + (tid>>3) + 32i, k quad tid&7 (like A)
#pragma unroll
      for (int i = 0; i < FB_N; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        boff[i] = n < g.N ? (n * g.K + 4 * (tid & 7)) * 4 : OOB;
      }
      f_cin = g.fC.d;
      f_tap = kbeg / f_cin;
      f_c0 = kbeg - f_tap * f_cin;
    } else {
      const int m = m0 + 4 * sw_q(BM);
#pragma unroll
      for (int i = 0; i < FA_N; ++i) aoff[i] = m < g.M ? (sw_p(BM, i) * (int)g.a.sw + m) * 4 : OOB;
      // the block's n tile lies in one tap: n0 -> (kh, kw, ci0), wave-uniform
      const uint32_t t = g.fC.div(n0);
      const int ci0 = n0 - t * g.fC.d;
      const uint32_t kh = g.fKW.div(t);
      const int kw = t - kh * g.fKW.d;
      w_tab = ((int)kh - g.pad) * (int)g.im.sh + ((int)kw - g.pad) * (int)g.im.sw + ci0;  // tap part
      f_tap = (int)kh;   // kept for the bounds checks below
      f_c0 = kw;
      // column quad of this thread's B loads -> (tap within the tile, channel): with
      // Cin >= BN every quad is in the first tap (4 q < BN <= Cin)
      const int cin = (int)g.fC.d, c4 = 4 * sw_q(BN);
      w_ntap = cin >= BN ? 1 : BN / cin;
      w_tq = cin >= BN ? 0 : c4 / cin;
      w_qb = (c4 - w_tq * cin) * 4;
    }
  }
  // CONV/CONVT2 FAST: per-row offsets for the current tap
  auto set_tap = [&](int tap) {
    if constexpr (FAST && MODE != MODE_WGRAD) {
      int dh, dw;
      if constexpr (MODE == MODE_CONV) {
        dh = tap / g.KW;
        dw = tap - dh * g.KW;
      } else {
        dh = ph - (tap >> 1);
        dw = pw - (tap & 1);
      }
      const int q = tid & 7;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int ih = aih[i] + dh, iw = aiw[i] + dw;
        aoff[i] = ((unsigned)ih < (unsigned)g.a.H && (unsigned)iw < (unsigned)g.a.W)
                      ? ((int)abase[i] + ih * (int)g.a.sh + iw * (int)g.a.sw) * 4 + q * 16
                      : OOB;
      }
    }
  };
  // WGRAD FAST: one wave writes the im2col pixel offsets of tile k0 into ptab[slot], for
  // each of the tile's taps (kw0 + t of kernel row kh)
  auto build_table = [&](int k0, int slot) {
    if constexpr (FAST && MODE == MODE_WGRAD) {
      const int l = tid & 63;
      if (l < BK) {
        const int p = k0 + l;
        const uint32_t b = g.fghw.div(p);
        const uint32_t rem = p - b * g.fghw.d;
        const uint32_t oi = g.fgw.div(rem);
        const uint32_t oj = rem - oi * g.fgw.d;
        const int ih = (int)oi * g.stride - g.pad + f_tap;
        const int pix = (int)b * (int)g.im.sb + (int)oi * g.stride * (int)g.im.sh + (int)oj * g.stride * (int)g.im.sw;
        const bool rok = p < kend && (unsigned)ih < (unsigned)g.im.H;
        for (int t = 0; t < w_ntap; ++t) {
          const int iw = (int)oj * g.stride - g.pad + f_c0 + t;
          ptab[slot][t * BK + l] =
              (rok && (unsigned)iw < (unsigned)g.im.W) ? (pix + w_tab + t * (int)g.im.sw) * 4 : OOB;
        }
      }
    }
  };
  auto load_fast = [&](int k0, int slot) {
    if constexpr (FAST && MODE != MODE_WGRAD) {
      if (f_c0 == f_cin) {
        f_c0 = 0;
        set_tap(++f_tap);
      }
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(arsrc, aoff[i], f_c0 * 4, 0);
        ra[4 * i + 0] = __uint_as_float(v.x); ra[4 * i + 1] = __uint_as_float(v.y);
        ra[4 * i + 2] = __uint_as_float(v.z); ra[4 * i + 3] = __uint_as_float(v.w);
      }
      f_c0 += BK;
      const int so = k0 * 4;
#pragma unroll
      for (int i = 0; i < FB_N; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff[i], so, 0);
        rb[4 * i + 0] = __uint_as_float(v.x); rb[4 * i + 1] = __uint_as_float(v.y);
        rb[4 * i + 2] = __uint_as_float(v.z); rb[4 * i + 3] = __uint_as_float(v.w);
      }
    } else if constexpr (FAST) {
      st_k0 = k0;
      const int so = k0 * (int)g.a.sw * 4;
#pragma unroll
      for (int i = 0; i < FA_N; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(arsrc, aoff[i], so, 0);
        ra[4 * i + 0] = __uint_as_float(v.x); ra[4 * i + 1] = __uint_as_float(v.y);
        ra[4 * i + 2] = __uint_as_float(v.z); ra[4 * i + 3] = __uint_as_float(v.w);
      }
#pragma unroll
      for (int i = 0; i < FB_N; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(brsrc, ptab[slot][w_tq * BK + sw_p(BN, i)] + w_qb, 0, 0);
        rb[4 * i + 0] = __uint_as_float(v.x); rb[4 * i + 1] = __uint_as_float(v.y);
        rb[4 * i + 2] = __uint_as_float(v.z); rb[4 * i + 3] = __uint_as_float(v.w);
      }
    }
  };

  auto load_tiles = [&](int k0) {
    // ---------------- A ----------------
    if constexpr (MODE != MODE_WGRAD) {
      if constexpr (AV) {
        const int q = tid & 7;
        const int k = k0 + 4 * q;
        int dh = 0, dw = 0, ci = 0;
        const bool kok = k < kend;
        if (kok) {
          uint32_t t = g.fC.div(k);
          ci = k - t * g.fC.d;
          if constexpr (MODE == MODE_CONV) {
            uint32_t kh = g.fKW.div(t);
            dh = kh;
            dw = t - kh * g.fKW.d;
          } else {
            int th = t >> 1, tw = t & 1;
            dh = ph - th;
            dw = pw - tw;
          }
        }
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          int ih = aih[i] + dh, iw = aiw[i] + dw;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (kok && (unsigned)ih < (unsigned)g.a.H && (unsigned)iw < (unsigned)g.a.W)
            v = *reinterpret_cast<const float4*>(g.a.p + abase[i] + (long long)ih * g.a.sh +
                                                 (long long)iw * g.a.sw + ci);
          ra[4 * i + 0] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < A_ELEMS; ++j) {
          int e = tid + 256 * j;
          int row = e >> 5, col = e & 31;
          int m = m0 + row, k = k0 + col;
          float v = 0.f;
          if (m < g.M && k < kend) {
            uint32_t b = g.fghw.div(m);
            uint32_t rem = m - b * g.fghw.d;
            uint32_t oi = g.fgw.div(rem);
            uint32_t oj = rem - oi * g.fgw.d;
            uint32_t t = g.fC.div(k);
            int ci = k - t * g.fC.d;
            int ih, iw;
            if constexpr (MODE == MODE_CONV) {
              uint32_t kh = g.fKW.div(t);
              ih = (int)oi * g.stride - g.pad + (int)kh;
              iw = (int)oj * g.stride - g.pad + (int)(t - kh * g.fKW.d);
            } else {
              ih = (int)oi + ph - (int)(t >> 1);
              iw = (int)oj + pw - (int)(t & 1);
            }
            if ((unsigned)ih < (unsigned)g.a.H && (unsigned)iw < (unsigned)g.a.W)
              v = g.a.p[(long long)b * g.a.sb + (long long)ih * g.a.sh + (long long)iw * g.a.sw +
                        (long long)ci * g.a.sc];
          }
          ra[j] = v;
        }
      }
    } else {
      // WGRAD A: rows p (k dim), cols m (gradient channel)
      if constexpr (AV) {
        constexpr int TPR = BM / 4, RPP = 256 / TPR, PASSES = BK / RPP;
        const int q = tid % TPR, r = tid / TPR;
        const int m = m0 + 4 * q;
#pragma unroll
        for (int i = 0; i < PASSES; ++i) {
          int p = k0 + r + RPP * i;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (p < kend && m < g.M) {
            uint32_t b = g.fghw.div(p);
            uint32_t rem = p - b * g.fghw.d;
            uint32_t oi = g.fgw.div(rem);
            uint32_t oj = rem - oi * g.fgw.d;
            v = *reinterpret_cast<const float4*>(g.a.p + (long long)b * g.a.sb + (long long)oi * g.a.sh +
                                                 (long long)oj * g.a.sw + m);
          }
          ra[4 * i + 0] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < A_ELEMS; ++j) {
          int e = tid + 256 * j;
          int row = e / BM, col = e - (e / BM) * BM;
          int p = k0 + row, m = m0 + col;
          float v = 0.f;
          if (p < kend && m < g.M) {
            uint32_t b = g.fghw.div(p);
            uint32_t rem = p - b * g.fghw.d;
            uint32_t oi = g.fgw.div(rem);
            uint32_t oj = rem - oi * g.fgw.d;
            v = g.a.p[(long long)b * g.a.sb + (long long)oi * g.a.sh + (long long)oj * g.a.sw +
                      (long long)m * g.a.sc];
          }
          ra[j] = v;
        }
      }
    }
    // ---------------- B ----------------
    if constexpr (MODE != MODE_WGRAD) {
      // packed weights [N][K]: k fastest across threads (coalesced), staged [k][n]
#pragma unroll
      for (int j = 0; j < B_ELEMS; ++j) {
        int e = tid + 256 * j;
        int row = e / BK, col = e - row * BK;
        int k = k0 + col, n = n0 + row;
        rb[j] = (k < kend && n < g.N) ? Bw[(size_t)n * g.K + k] : 0.f;
      }
    } else {
      // WGRAD B: im2col(img)[p][n]
      if constexpr (BV) {
        constexpr int TPR = BN / 4, RPP = 256 / TPR, PASSES = BK / RPP;
        const int r = tid / TPR;
#pragma unroll
        for (int i = 0; i < PASSES; ++i) {
          int p = k0 + r + RPP * i;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (p < kend && wb_nok) {
            uint32_t b = g.fghw.div(p);
            uint32_t rem = p - b * g.fghw.d;
            uint32_t oi = g.fgw.div(rem);
            uint32_t oj = rem - oi * g.fgw.d;
            int ih = (int)oi * g.stride - g.pad + wb_kh;
            int iw = (int)oj * g.stride - g.pad + wb_kw;
            if ((unsigned)ih < (unsigned)g.im.H && (unsigned)iw < (unsigned)g.im.W)
              v = *reinterpret_cast<const float4*>(g.im.p + (long long)b * g.im.sb + (long long)ih * g.im.sh +
                                                   (long long)iw * g.im.sw + wb_ci);
          }
          rb[4 * i + 0] = v.x; rb[4 * i + 1] = v.y; rb[4 * i + 2] = v.z; rb[4 * i + 3] = v.w;
        }
      } else {
        if (g.im_buf) {
          // every gather unconditional, a tap outside the image at an offset past the
          // descriptor (reads 0): a conditional load compiles into a branch that waits for it
          // -- one gather in flight per thread (round 6: C4's input-layer weight gradient)
#pragma unroll
          for (int j = 0; j < B_ELEMS; ++j) {
            const int e = tid + 256 * j, row = e / BN, col = e - row * BN, p = k0 + row, n = n0 + col;
            const bool in = p < kend && n < g.N;
            const uint32_t b = g.fghw.div(p), rem = p - b * g.fghw.d, oi = g.fgw.div(rem), oj = rem - oi * g.fgw.d;
            const uint32_t t = g.fC.div(n), kh = g.fKW.div(t);
            const int ci = n - t * g.fC.d, kw = t - kh * g.fKW.d;
            const int ih = (int)oi * g.stride - g.pad + (int)kh, iw = (int)oj * g.stride - g.pad + kw;
            const bool ok = in && (unsigned)ih < (unsigned)g.im.H && (unsigned)iw < (unsigned)g.im.W;
            const int off = (int)b * (int)g.im.sb + ih * (int)g.im.sh + iw * (int)g.im.sw + ci * (int)g.im.sc;
            rb[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brsrc, ok ? 4 * off : 0x7ffffff0, 0, 0));
          }
        } else {
#pragma unroll
          for (int j = 0; j < B_ELEMS; ++j) {
            int e = tid + 256 * j;
            int row = e / BN, col = e - (e / BN) * BN;
            int p = k0 + row, n = n0 + col;
            float v = 0.f;
            if (p < kend && n < g.N) {
              uint32_t b = g.fghw.div(p);
              uint32_t rem = p - b * g.fghw.d;
              uint32_t oi = g.fgw.div(rem);
              uint32_t oj = rem - oi * g.fgw.d;
              uint32_t t = g.fC.div(n);
              int ci = n - t * g.fC.d;
              uint32_t kh = g.fKW.div(t);
              int kw = t - kh * g.fKW.d;
              int ih = (int)oi * g.stride - g.pad + (int)kh;
              int iw = (int)oj * g.stride - g.pad + kw;
              if ((unsigned)ih < (unsigned)g.im.H && (unsigned)iw < (unsigned)g.im.W)
                v = g.im.p[(long long)b * g.im.sb + (long long)ih * g.im.sh + (long long)iw * g.im.sw +
                           (long long)ci * g.im.sc];
            }
            rb[j] = v;
          }
        }
      }
    }
  };

  // bias gradient of a FAST conv WGRAD (GemmArgs::dbias): this thread's 4 channels (m0 + 4 q
  // .. + 3, q = sw_q(BM)) summed in double over the pixels it stages
  const bool db_on = SWZ && g.dbias != nullptr && tn_i == 0;
  double dbs[4] = {0.0, 0.0, 0.0, 0.0};
  auto store_tiles = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + A_SZ;
    if constexpr (SWZ) {
      if (db_on && st_k0 >= g.db_k0) {  // tile-uniform: db_k0 is a multiple of BK
#pragma unroll
        for (int i = 0; i < FA_N; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) dbs[j] += (double)ra[4 * i + j];
      }
      // element (row, k) at row * 32 + 4 ((k >> 2) ^ ((row >> 1) & 7)) + (k & 3)
      auto put = [&](float* T, int R, const float* v, int nld) {
        const int q = sw_q(R);
#pragma unroll
        for (int i = 0; i < nld; ++i) {
          const int k = sw_p(R, i);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = 4 * q + j;
            T[row * KROW_LD + 4 * ((k >> 2) ^ ((row >> 1) & 7)) + (k & 3)] = v[4 * i + j];
          }
        }
      };
      put(As, BM, ra, FA_N);
      put(Bs, BN, rb, FB_N);
      return;
    } else if constexpr (KROW) {
      const int q = tid & 7;
#pragma unroll
      for (int i = 0; i < AR; ++i)
        *reinterpret_cast<float4*>(As + ((tid >> 3) + 32 * i) * KROW_LD + 4 * q) =
            make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]);
#pragma unroll
      for (int i = 0; i < FB_N; ++i)
        *reinterpret_cast<float4*>(Bs + ((tid >> 3) + 32 * i) * KROW_LD + 4 * q) =
            make_float4(rb[4 * i], rb[4 * i + 1], rb[4 * i + 2], rb[4 * i + 3]);
      return;
    }
    if constexpr (MODE != MODE_WGRAD) {
      if constexpr (AV) {
        const int q = tid & 7;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          float* dst = As + ((tid >> 3) + 32 * i) * A_LD + 4 * q;
          dst[0] = ra[4 * i + 0]; dst[1] = ra[4 * i + 1]; dst[2] = ra[4 * i + 2]; dst[3] = ra[4 * i + 3];
        }
      } else {
#pragma unroll
        for (int j = 0; j < A_ELEMS; ++j) {
          int e = tid + 256 * j;
          As[(e >> 5) * A_LD + (e & 31)] = ra[j];
        }
      }
    } else {
      if constexpr (AV) {
        constexpr int TPR = BM / 4, RPP = 256 / TPR, PASSES = BK / RPP;
        const int q = tid % TPR, r = tid / TPR;
#pragma unroll
        for (int i = 0; i < PASSES; ++i)
          *reinterpret_cast<float4*>(As + (r + RPP * i) * A_LD + 4 * q) =
              make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]);
      } else {
#pragma unroll
        for (int j = 0; j < A_ELEMS; ++j) {
          int e = tid + 256 * j;
          int row = e / BM;
          As[row * A_LD + (e - row * BM)] = ra[j];
        }
      }
    }
    if constexpr (MODE != MODE_WGRAD) {  // [N][K] weights, k fastest (load_tiles)
#pragma unroll
      for (int j = 0; j < B_ELEMS; ++j) {
        int e = tid + 256 * j;
        int row = e / BK;
        Bs[(e - row * BK) * B_LD + row] = rb[j];
      }
    } else if constexpr (BV) {
      constexpr int TPR = BN / 4, RPP = 256 / TPR, PASSES = BK / RPP;
      const int q = tid % TPR, r = tid / TPR;
#pragma unroll
      for (int i = 0; i < PASSES; ++i)
        *reinterpret_cast<float4*>(Bs + (r + RPP * i) * B_LD + 4 * q) =
            make_float4(rb[4 * i], rb[4 * i + 1], rb[4 * i + 2], rb[4 * i + 3]);
    } else {
#pragma unroll
      for (int j = 0; j < B_ELEMS; ++j) {
        int e = tid + 256 * j;
        int row = e / BN;
        Bs[row * B_LD + (e - row * BN)] = rb[j];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // vector epilogue's per-tile output row offsets (FAST 64x64-per-wave tiles)
  constexpr bool VEC_EPI = KROW && BM / WM == 64 && BN / WN == 64;
  __shared__ long long emoff[VEC_EPI ? BM : 1];
  // Producer post-op (gemm_post: unsplit tiles, vector epilogue): the rows of px the epilogue
  // multiplies by are loaded into registers at the start of the LAST k tile, so their HBM
  // latency hides under that tile's MFMAs instead of stalling the epilogue.  The row-offset
  // table they index is written here, at the start, and published by the main loop's barriers.
  float4 pax[VEC_EPI && POST ? 16 : 1];
  const bool post_pf = POST && VEC_EPI && g.pmode && g.splits == 1 && g.vec_out;
  if constexpr (POST && VEC_EPI) {
    if (post_pf) {
      for (int i = tid; i < BM; i += 256) {
        const int m = m0 + i;
        emoff[i] = m < g.M ? row_offset(g.out, m, MODE == MODE_CONVT2 ? phase : 0) : 0;
      }
    }
  }
  auto post_prefetch = [&]() {
    if constexpr (POST && VEC_EPI) {
      const int n = n0 + wn + 4 * (lane & 15);
      if (post_pf && n < g.N) {
        const long long noff = col_offset(g.out, n);
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
          const int rl = 4 * s4 + (lane >> 4), m = m0 + wm + rl;
          pax[s4] = m < g.M ? *reinterpret_cast<const float4*>(g.px + emoff[wm + rl] + noff)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  };

  if constexpr (FAST && MODE == MODE_WGRAD) {
    if (wid == 0) build_table(kbeg, 0);
    if (wid == 1 && nk > 1) build_table(kbeg + BK, 1);
    __syncthreads();
  }
  if constexpr (FAST && MODE != MODE_WGRAD) set_tap(f_tap);
  const int l32 = lane & 31, lk = lane >> 5;
  if constexpr (EMU) {
    // fp32 GEMM on the bf16 MFMA: every operand is split EXACTLY into three bf16 pieces
    // (x = hi + mid + lo, 8 significant bits each: hi = x with the low 16 bits cleared,
    // mid likewise of x - hi, lo = x - hi - mid, exact in bf16), and each product keeps the
    // six terms down to 2^-16 relative: hh, hm, mh, hl, lh, mm (bf16 x bf16 products are
    // exact in fp32; the dropped ml, lm, ll terms are <= 2^-23 relative -- one fp32
    // rounding).  v_mfma_f32_32x32x16_bf16 has 16x the rate of the fp32 MFMA, so 6 of them
    // are 2.67x fewer MFMA cycles; the split (about 6 VALU per element) overlaps the bf16
    // MFMAs, which -- unlike fp32 MFMA -- co-execute with VALU.
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    uint32_t* P = reinterpret_cast<uint32_t*>(smem);  // planes 0-2 A, 3-5 B
    auto split_store = [&](uint32_t* base, int row, int q, const float* v) {
      uint32_t h[4], m[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t xb = __float_as_uint(v[e]);
        h[e] = xb & 0xffff0000u;
        const float r1 = v[e] - __uint_as_float(h[e]);
        m[e] = __float_as_uint(r1) & 0xffff0000u;
        l[e] = __float_as_uint(r1 - __uint_as_float(m[e]));
      }
      const int o = row * EMU_RS + 2 * q;  // k 4q .. 4q+3 = dwords 2q, 2q+1 of the row
      *reinterpret_cast<uint2*>(base + o) = make_uint2((h[0] >> 16) | h[1], (h[2] >> 16) | h[3]);
      *reinterpret_cast<uint2*>(base + EMU_PLANE + o) = make_uint2((m[0] >> 16) | m[1], (m[2] >> 16) | m[3]);
      *reinterpret_cast<uint2*>(base + 2 * EMU_PLANE + o) =
          make_uint2((l[0] >> 16) | (l[1] & 0xffff0000u), (l[2] >> 16) | (l[3] & 0xffff0000u));
    };
    auto store_emu = [&]() {
      const int q = tid & 7;
#pragma unroll
      for (int i = 0; i < AR; ++i) split_store(P, (tid >> 3) + 32 * i, q, ra + 4 * i);
#pragma unroll
      for (int i = 0; i < FB_N; ++i) split_store(P + 3 * EMU_PLANE, (tid >> 3) + 32 * i, q, rb + 4 * i);
    };
    if (nk > 0) {
      load_fast(kbeg, 0);
      store_emu();
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      // registers only, in flight during the MFMAs.  Unconditional: a guarded load leaves
      // the compiler a phi of (new, old) registers whose copies wait for the loads right
      // here.  Past the last tile every offset is in-bounds or OOB (buffer loads return 0).
      load_fast(kbeg + (kt + 1) * BK, 0);
      if (kt + 1 == nk) post_prefetch();
      __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs (not sunk for VGPRs)
#pragma unroll
      for (int t = 0; t < 2; ++t) {  // two k16 steps per BK = 32 tile; lane half lk takes k 8 lk .. 8 lk + 7
        bf16x8 af[3][TM], bfr[3][TN];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            af[pl][i] = *reinterpret_cast<const bf16x8*>(P + pl * EMU_PLANE + (wm + 32 * i + l32) * EMU_RS + 8 * t + 4 * lk);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            bfr[pl][j] = *reinterpret_cast<const bf16x8*>(P + (3 + pl) * EMU_PLANE + (wn + 32 * j + l32) * EMU_RS +
                                                          8 * t + 4 * lk);
        }
        // (A first: rows of the product are pixels, columns output channels, as in the fp32 path)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x16 c = acc[i][j];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bfr[2][j], c, 0, 0, 0);  // A hi x B lo
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][i], bfr[0][j], c, 0, 0, 0);  // A lo x B hi
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bfr[1][j], c, 0, 0, 0);  // A mid x B mid
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bfr[1][j], c, 0, 0, 0);  // A hi x B mid
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bfr[0][j], c, 0, 0, 0);  // A mid x B hi
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bfr[0][j], c, 0, 0, 0);  // A hi x B hi
          }
      }
      __syncthreads();  // every wave's reads of this tile are done
      if (kt + 1 < nk) {
        store_emu();
        __syncthreads();
      }
    }
  } else {
  if (nk > 0) {
    if constexpr (FAST) load_fast(kbeg, 0);
    else load_tiles(kbeg);
    store_tiles(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = GEMM_SB ? 0 : kt & 1;
    if (kt + 1 < nk) {
      if constexpr (FAST) load_fast(kbeg + (kt + 1) * BK, (kt + 1) & 1);
      else load_tiles(kbeg + (kt + 1) * BK);
    } else {
      post_prefetch();
    }
    if constexpr (FAST && MODE == MODE_WGRAD) {
      if (kt + 2 < nk && wid == (kt & 3)) build_table(kbeg + (kt + 2) * BK, kt & 1);
    }
    const float* As = smem + cur * STAGE;
    const float* Bs = As + A_SZ;
    if constexpr (KROW) {
      // logical quad g = kq + 4 lk of row wm/wn + 32 t + l32; SWZ: physical quad g ^ swz
      // with swz = (l32 >> 1) & 7 (wm, wn, 32 t are multiples of 32)
      const int swz = SWZ ? (l32 >> 1) & 7 : 0;
      const float* Ar = As + (wm + l32) * KROW_LD;
      const float* Br = Bs + (wn + l32) * KROW_LD;
#pragma unroll
      for (int kq = 0; kq < BK / 8; ++kq) {
        const int qo = 4 * ((kq + 4 * lk) ^ swz);
        float4 a4[TM], b4[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) a4[t] = *reinterpret_cast<const float4*>(Ar + 32 * t * KROW_LD + qo);
#pragma unroll
        for (int t = 0; t < TN; ++t) b4[t] = *reinterpret_cast<const float4*>(Br + 32 * t * KROW_LD + qo);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i][s4], b4[j][s4], acc[i][j], 0, 0, 0);
      }
    } else {
    // per-lane base pointers: every operand read below is base + compile-time offset,
    // which folds into the DS instruction's immediate (no per-read address VALU)
    const float* Al = AK ? As + lk * A_LD + wm + l32 : As + (wm + l32) * A_LD + lk;
    const float* Bl = Bs + lk * B_LD + wn + l32;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      float af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = AK ? Al[2 * kk * A_LD + 32 * t] : Al[32 * t * A_LD + 2 * kk];
#pragma unroll
      for (int t = 0; t < TN; ++t) bf[t] = Bl[2 * kk * B_LD + 32 * t];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    }
    if constexpr (GEMM_SB) {
      if (kt + 1 < nk) {
        __syncthreads();  // every wave's reads of the one stage are done
        store_tiles(0);
      }
    } else if (kt + 1 < nk) {
      store_tiles(cur ^ 1);
    }
    __syncthreads();
  }
  }  // EMU / fp32 main loop

  const bool split_out = g.splits > 1;  // partial sums for a separate splitk_reduce

  if constexpr (SWZ) {
    if (db_on) {
      // the NT8 = 1024 / BM threads staging the same channel quad (pixel slots t8 =
      // ((tid >> 3) & 3) + 4 ((tid >> 5) / (BM / 32)): 8 slots for 128-row tiles, 16 for the
      // 64-row ones) -> one double per channel, t8 in order (the main loop's last barrier has
      // retired every stage read; the epilogue reuses smem after the second barrier)
      double* dsh = reinterpret_cast<double*>(smem);
      constexpr int NT8 = 1024 / BM;  // threads staging one channel quad
      const int q = sw_q(BM), t8 = ((tid >> 3) & 3) + 4 * ((tid >> 5) / (BM / 32));
#pragma unroll
      for (int j = 0; j < 4; ++j) dsh[t8 * BM + 4 * q + j] = dbs[j];
      __syncthreads();
      if (tid < BM && m0 + tid < g.M) {
        double v = 0.0;
#pragma unroll
        for (int t = 0; t < NT8; ++t) v += dsh[t * BM + tid];
        if (split_out) {
          g.dbp[(size_t)split * g.M + m0 + tid] = v;
        } else {
          float* dst = g.dbias + m0 + tid;
          *dst = g.db_accum ? *dst + (float)v : (float)v;
        }
      }
      __syncthreads();
    }
  }

  // ---------------- epilogue ----------------
  if constexpr (VEC_EPI) {
    // Vector epilogue (FAST, 64x64 per wave): each wave stages its finished sub-tile in LDS
    // (row stride 72: the two lane halves' rows 4 apart land 32 banks apart) and writes it
    // back as float4 rows -- 16 b128 stores per lane instead of 64 scalar ones, 256
    // contiguous bytes per output row.  The scalar stores' bursts at the end of every tile
    // (all blocks finish together) held the MFMA pipes idle on short-K layers.
    const bool slab_out = split_out;
    if ((slab_out && g.N % 4 == 0) || (!slab_out && g.vec_out)) {
      constexpr int EP_LD = 72, EPR = GEMM_SB ? 32 : 64, NP = 64 / EPR;
      float* T = smem + wid * (EPR * EP_LD);
      const float wsc = (!slab_out && g.wscale) ? g.wscale[0] : 1.f;
      if (!slab_out && !post_pf) {
        for (int i = tid; i < BM; i += 256) {
          const int m = m0 + i;
          emoff[i] = m < g.M ? row_offset(g.out, m, MODE == MODE_CONVT2 ? phase : 0) : 0;
        }
      }
      // the activation branch is taken once per tile (uniform), not once per element
      auto stage = [&](auto actf, int pp) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cl = 32 * j + l32, col = n0 + wn + cl;
          const float bv = (!slab_out && g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            if (NP > 1 && i != pp) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk - EPR * pp;
              T[rl * EP_LD + cl] = actf(acc[i][j][r] * wsc + bv);
            }
          }
        }
      };
      const bool bn_stats = !slab_out && g.bnp;
      double s1 = 0.0, s2 = 0.0;
      const int q = lane & 15, n = n0 + wn + 4 * q;
      float* slab = slab_out ? g.slab + (size_t)z * g.M * g.N : nullptr;
      const long long noff = (slab_out || n >= g.N) ? 0 : col_offset(g.out, n);
      // producer post-op (unsplit only; the reduce applies it to split tiles).  pmode 2: the
      // wave's 64 rows are one 64-row segment of one batch segment (host: bn_post_ok)
      const int pmode = (!POST || slab_out) ? 0 : g.pmode;
      float p_al[4], p_be[4], p_mu[4];
      double p1[4] = {0.0, 0.0, 0.0, 0.0}, p2[4] = {0.0, 0.0, 0.0, 0.0};
      if (pmode == 2) {
        const int k = post_seg(g, m0 + wm);
#pragma unroll
        for (int i = 0; i < 4; ++i) post_consts(g, k, n + i, p_al[i], p_be[i], p_mu[i]);
      }
#pragma unroll
      for (int pp = 0; pp < NP; ++pp) {
        if (pp > 0) __syncthreads();  // the previous pass's T reads are done
        if (slab_out || g.act <= RGAN_ACT_LRELU) {
          const float neg = (slab_out || g.act == RGAN_ACT_NONE) ? 1.f : (g.act == RGAN_ACT_RELU ? 0.f : g.alpha);
          stage([neg](float v) { return v > 0.f ? v : v * neg; }, pp);
        } else {
          stage([&](float v) { return act_fwd_curved(v, g.act, g.alpha); }, pp);
        }
        __syncthreads();
        if (bn_stats) {
          // BatchNorm batch statistics in the epilogue: the wave's finished rows of column
          // `lane` (one channel; conflict-free LDS row reads) -> (sum y, sum y^2) of the
          // 64-row segment in double, rows in order (fp32 products are exact in double; the
          // merge is a plain fixed-order sum).  Host guarantees M % 64 == 0 and n == channel;
          // segment = (phase, m / 64).
#pragma unroll 8
          for (int rl = 0; rl < EPR; ++rl) {
            const double d = (double)T[rl * EP_LD + lane];
            s1 += d;
            s2 += d * d;
          }
        }
        if (n < g.N && pmode) {
          // producer post-op: the wave's 16 rows of px, loaded during the last k tile
          // (post_prefetch; GEMM_SB is off for these 128x128 tiles: one pass, pp = 0)
          static_assert(!POST || EPR == 64, "post-op prefetch covers one 64-row pass");
          const float4* ax = pax;
#pragma unroll
          for (int s4 = 0; s4 < EPR / 4; ++s4) {
            const int rl = 4 * s4 + (lane >> 4), m = m0 + wm + EPR * pp + rl;
            if (m < g.M) {
              const float4 v = *reinterpret_cast<const float4*>(T + rl * EP_LD + 4 * q);
              float vv[4] = {v.x, v.y, v.z, v.w};
              const float aa[4] = {ax[s4].x, ax[s4].y, ax[s4].z, ax[s4].w};
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                if (pmode == 1) {
                  vv[i] *= act_grad_from_out(aa[i], g.pact, g.palpha);
                } else {
                  vv[i] *= act_grad_from_in(aa[i] * p_al[i] + p_be[i], g.pact, g.palpha);
                  p1[i] += (double)vv[i];
                  p2[i] += (double)vv[i] * (double)(aa[i] - p_mu[i]);
                }
              }
              *reinterpret_cast<float4*>(g.C + emoff[wm + EPR * pp + rl] + noff) = make_float4(vv[0], vv[1], vv[2], vv[3]);
            }
          }
        } else if (n < g.N) {
#pragma unroll
          for (int s4 = 0; s4 < EPR / 4; ++s4) {
            const int rl = 4 * s4 + (lane >> 4), m = m0 + wm + EPR * pp + rl;
            if (m < g.M) {
              const float4 v = *reinterpret_cast<const float4*>(T + rl * EP_LD + 4 * q);
              float* dst = slab_out ? slab + (size_t)m * g.N + n : g.C + emoff[wm + EPR * pp + rl] + noff;
              *reinterpret_cast<float4*>(dst) = v;
            }
          }
        }
      }
      if (bn_stats) {
        const int mrow = m0 + wm, col = n0 + wn + lane;
        if (mrow < g.M && col < g.N) {
          const size_t seg = (size_t)phase * (uint32_t)(g.M >> 6) + (uint32_t)(mrow >> 6);
          g.bnp[(seg * 2) * g.N + col] = s1;
          g.bnp[(seg * 2 + 1) * g.N + col] = s2;
        }
      }
      if (pmode == 2) {
        // the 4 row groups (lane >> 4) of each column quad: fixed xor-butterfly (a + b == b + a
        // bitwise, so every lane of a group ends with the same sums)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p1[i] += __shfl_xor(p1[i], 16);
          p2[i] += __shfl_xor(p2[i], 16);
          p1[i] += __shfl_xor(p1[i], 32);
          p2[i] += __shfl_xor(p2[i], 32);
        }
        const int mrow = m0 + wm;
        if ((lane >> 4) == 0 && mrow < g.M) {
          const size_t seg = (size_t)phase * (uint32_t)(g.M >> 6) + (uint32_t)(mrow >> 6);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (n + i < g.N) {
              g.ppart[(seg * 2) * g.N + n + i] = p1[i];
              g.ppart[(seg * 2 + 1) * g.N + n + i] = p2[i];
            }
          }
        }
      }
      return;
    }
  }
  if (split_out) {
    float* slab = g.slab + (size_t)z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn + 32 * j + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (row < g.M && col < g.N) slab[(size_t)row * g.N + col] = acc[i][j][r];
        }
      }
    return;
  }
  const float wsc = g.wscale ? g.wscale[0] : 1.f;
  long long* moff = reinterpret_cast<long long*>(smem);
  long long* noff = moff + BM;
  for (int i = tid; i < BM; i += 256) {
    int m = m0 + i;
    moff[i] = m < g.M ? row_offset(g.out, m, MODE == MODE_CONVT2 ? phase : 0) : 0;
  }
  for (int i = tid; i < BN; i += 256) {
    int n = n0 + i;
    noff[i] = n < g.N ? col_offset(g.out, n) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn + 32 * j + l32;
      const int col = n0 + cl;
      const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
      auto put = [&](auto actf) {
        if constexpr (MODE == MODE_WGRAD) {
          // accumulating: the 16 old values first, all in flight, through a descriptor over
          // dW (rows outside the tile at an offset past it) -- the read-modify-write per
          // element compiled into 16 dependent round trips
          if (g.accum && (long long)g.M * g.N * 4 < 0x7ffffff0LL) {
            const __amdgpu_buffer_rsrc_t crs =
                __builtin_amdgcn_make_buffer_rsrc((void*)g.C, (short)0, (int)(4LL * g.M * g.N), 0x00020000);
            float old[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
              const bool ok = m0 + rl < g.M && col < g.N;
              old[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  crs, ok ? (int)(4 * (moff[rl] + noff[cl])) : 0x7ffffff0, 0, 0));
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
              if (m0 + rl < g.M && col < g.N) g.C[moff[rl] + noff[cl]] = old[r] + actf(acc[i][j][r] * wsc + bv);
            }
            return;
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (m0 + rl < g.M && col < g.N) {
            float v = acc[i][j][r] * wsc + bv;
            float* dst = g.C + moff[rl] + noff[cl];
            v = actf(v);
            *dst = (MODE == MODE_WGRAD && g.accum) ? *dst + v : v;
          }
        }
      };
      if (g.act <= RGAN_ACT_LRELU) {
        const float neg = g.act == RGAN_ACT_NONE ? 1.f : (g.act == RGAN_ACT_RELU ? 0.f : g.alpha);
        put([neg](float v) { return v > 0.f ? v : v * neg; });
      } else {
        put([&](float v) { return act_fwd_curved(v, g.act, g.alpha); });
      }
    }
  if constexpr (BM == 64 && BN == 64 && MODE != MODE_WGRAD) {
    if (g.bnp) {
      // BatchNorm segment sums of the 64 x 64 tile (unsplit, act none, n = channel, M % 64 ==
      // 0: host bn_epilogue_ok): the tile's 64 rows are one segment.  Per column: the lane's 16
      // rows in register order, then the two lane halves (xor 32), then the two waves of the
      // column (wm = 0, 32) in order through LDS -- (sum y, sum y^2) in double of the values
      // stored above, as the 128 x 128 vector epilogue writes them.
      double s1 = 0.0, s2 = 0.0;
      const int cl = wn + l32, col = n0 + cl;
      const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const double d = (double)(acc[0][0][r] * wsc + bv);
        s1 += d;
        s2 += d * d;
      }
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      double* bsh = reinterpret_cast<double*>(noff + BN);  // [2 waves][2][64]
      if (lk == 0) {
        bsh[(wm / 32) * 128 + cl] = s1;
        bsh[(wm / 32) * 128 + 64 + cl] = s2;
      }
      __syncthreads();
      if (tid < 64 && n0 + tid < g.N && m0 < g.M) {
        const size_t seg = (size_t)phase * (uint32_t)(g.M >> 6) + (uint32_t)(m0 >> 6);
        g.bnp[(seg * 2) * g.N + n0 + tid] = bsh[tid] + bsh[128 + tid];
        g.bnp[(seg * 2 + 1) * g.N + n0 + tid] = bsh[64 + tid] + bsh[192 + tid];
      }
    }
  }
}

template <int MODE, int BM, int BN, int WM, int WN, bool AV, bool BV, bool FAST>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs g) {
  gemm_body<MODE, BM, BN, WM, WN, AV, BV, FAST, false>(g);
}

// The FAST 128 x 128 CONV / CONVT2 GEMM with a producer post-op in its vector epilogue
// (GemmArgs::pmode, rgan_conv_post): its own instantiation, so the plain GEMMs' registers and
// schedule stay those of the post-free epilogue.
template <int MODE>
__global__ __launch_bounds__(256, 2) void gemm_post(GemmArgs g) {
  gemm_body<MODE, 128, 128, 2, 2, true, true, true, false, true>(g);
}
// ... and with the opt-in fp32-on-bf16x6 products (rgan_set_gemm_emulation)
template <int MODE>
__global__ __launch_bounds__(256, 2) void gemm_post_bf16x6(GemmArgs g) {
  gemm_body<MODE, 128, 128, 2, 2, true, true, true, true, true>(g);
}

// Opt-in (rgan_set_gemm_emulation): the FAST 128 x 128 CONV / CONVT2 GEMM with fp32 products
// emulated on the bf16 MFMA (see gemm_body's EMU path).  Its own symbol, reported as such.
template <int MODE>
__global__ __launch_bounds__(256, 2) void gemm_bf16x6(GemmArgs g) {
  gemm_body<MODE, 128, 128, 2, 2, true, true, true, true>(g);
}

// Split-K reduce: out = act(sum_sp slab[sp] * wscale + bias), slabs summed in split order
// (deterministic; loads issued 4 splits ahead of the adds).  Three shapes, chosen on the
// host:
//  RED_VEC  channel-contiguous outputs (tc == 1, 16-B aligned): one thread per (phase, m,
//           4 consecutive n), float4 loads and stores;
//  RED_TAPS torch weight layout (WGRAD, n = (kh, kw, c) over a 4x4 kernel, out[m][c][kh][kw]):
//           one thread per (m, c, 4 taps), 4 taps of a channel = one float4 store (lanes on
//           consecutive tap quads write contiguously);
//  RED_ANY  anything else, one element per thread.
enum { RED_ANY = 0, RED_VEC = 1, RED_TAPS = 2 };

__device__ __forceinline__ float red_epi(const GemmArgs& g, float v, float wsc, int n) {
  v *= wsc;
  if (g.bias) v += g.bias[n];
  return act_fwd(v, g.act, g.alpha);
}

// sum over splits of V-wide vectors at s + sp * stride, in split order
template <int V>
__device__ __forceinline__ void red_sum(const float* s, size_t stride, int splits, float (&v)[V]) {
  float t[4][V];
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = 0.f;
  int sp = 0;
  for (; sp + 4 <= splits; sp += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (V == 4) {
        const float4 q = *reinterpret_cast<const float4*>(s + (size_t)(sp + u) * stride);
        t[u][0] = q.x; t[u][1] = q.y; t[u][2] = q.z; t[u][3] = q.w;
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) t[u][i] = s[(size_t)(sp + u) * stride + i];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < V; ++i) v[i] = sp + u == 0 ? t[u][i] : v[i] + t[u][i];
  }
  for (; sp < splits; ++sp)
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = sp == 0 ? s[(size_t)sp * stride + i] : v[i] + s[(size_t)sp * stride + i];
}

// split FAST conv WGRAD with a bias: dbias[m] (+)= sum over splits of dbp[split][m] in split
// order (double), by the first block of the WGRAD reduce
__device__ __forceinline__ void wgrad_db_finish(const GemmArgs& g) {
  if (g.dbias == nullptr || blockIdx.x != 0 || blockIdx.y != 0) return;
  for (int m = threadIdx.x; m < g.M; m += blockDim.x) {
    double v = 0.0;
    for (int sp = 0; sp < g.splits; ++sp) v += g.dbp[(size_t)sp * g.M + m];
    g.dbias[m] = g.db_accum ? g.dbias[m] + (float)v : (float)v;
  }
}

template <int MODE, int KIND>
__global__ __launch_bounds__(256) void splitk_reduce(GemmArgs g, FastDiv fdiv, uint32_t per_phase) {
  if constexpr (MODE == MODE_WGRAD) wgrad_db_finish(g);
  const int phase = blockIdx.y;
  const size_t MN = (size_t)g.M * g.N;
  const float* base = g.slab + (size_t)phase * g.splits * MN;
  // the unsplit epilogue computes acc * wsc + bias; wsc = 1 multiplies exactly
  const float wsc = g.wscale ? g.wscale[0] : 1.f;
  for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < per_phase; idx += gridDim.x * 256u) {
    if constexpr (KIND == RED_VEC) {
      const uint32_t m = fdiv.div(idx);               // fdiv = N / 4
      const int n = 4 * (int)(idx - m * fdiv.d);
      float v[4];
      red_sum<4>(base + (size_t)m * g.N + n, MN, g.splits, v);
      float4 o = make_float4(red_epi(g, v[0], wsc, n), red_epi(g, v[1], wsc, n + 1),
                             red_epi(g, v[2], wsc, n + 2), red_epi(g, v[3], wsc, n + 3));
      const long long ooff = row_offset(g.out, (int)m, MODE == MODE_CONVT2 ? phase : 0) + col_offset(g.out, n);
      float4* dst = reinterpret_cast<float4*>(g.C + ooff);
      if (MODE != MODE_WGRAD && g.pmode == 1) {
        const float4 a = *reinterpret_cast<const float4*>(g.px + ooff);
        o.x *= act_grad_from_out(a.x, g.pact, g.palpha);
        o.y *= act_grad_from_out(a.y, g.pact, g.palpha);
        o.z *= act_grad_from_out(a.z, g.pact, g.palpha);
        o.w *= act_grad_from_out(a.w, g.pact, g.palpha);
      }
      if (g.accum) {
        const float4 q = *dst;
        *dst = make_float4(q.x + o.x, q.y + o.y, q.z + o.z, q.w + o.w);
      } else {
        *dst = o;
      }
    } else if constexpr (KIND == RED_TAPS) {
      const uint32_t mc = idx >> 2;                   // fdiv = channels c
      const int q = (int)(idx & 3);                   // taps 4q .. 4q+3 (kh = q)
      const uint32_t m = fdiv.div(mc);
      const int c = (int)(mc - m * fdiv.d);
      const float* s = base + (size_t)m * g.N + c;
      const int nc = (int)fdiv.d;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float w[1];
        red_sum<1>(s + (size_t)(4 * q + i) * nc, MN, g.splits, w);
        v[i] = red_epi(g, w[0], wsc, (4 * q + i) * nc + c);
      }
      float4* dst = reinterpret_cast<float4*>(g.C + (long long)m * g.out.sb + (long long)c * 16 + 4 * q);
      if (g.accum) {
        const float4 o = *dst;
        v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
      }
      *dst = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      const uint32_t m = fdiv.div(idx);               // fdiv = N
      const int n = (int)(idx - m * fdiv.d);
      float v[1];
      red_sum<1>(base + (size_t)m * g.N + n, MN, g.splits, v);
      const long long ooff = row_offset(g.out, (int)m, MODE == MODE_CONVT2 ? phase : 0) + col_offset(g.out, n);
      float* dst = g.C + ooff;
      float o = red_epi(g, v[0], wsc, n);
      if (MODE != MODE_WGRAD && g.pmode == 1) o *= act_grad_from_out(g.px[ooff], g.pact, g.palpha);
      *dst = g.accum ? *dst + o : o;
    }
  }
}

// RED_ANY shape with few outputs and many splits (the 1x1 patch GEMMs' weight gradients: a
// 128 x 64 output, split-K 512 ways): one thread per output would be a 512-long chain on
// 32 blocks.  Here a block = 16 outputs x 16 split lanes; lane l sums splits l, l + 16, ...
// in order (4 loads in flight), then a fixed LDS tree adds the 16 lane sums (deterministic;
// a different association than red_sum's split order, the same set of fp32 partials).
constexpr int REDW_OUT = 16, REDW_LANES = 16;
template <int MODE>
__global__ __launch_bounds__(256) void splitk_reduce_wide(GemmArgs g, FastDiv fdiv, uint32_t per_phase) {
  if constexpr (MODE == MODE_WGRAD) wgrad_db_finish(g);
  __shared__ float sh[REDW_LANES][REDW_OUT + 1];
  const int phase = blockIdx.y, ob = threadIdx.x % REDW_OUT, l = threadIdx.x / REDW_OUT;
  const size_t MN = (size_t)g.M * g.N;
  const uint32_t idx = blockIdx.x * REDW_OUT + ob;
  const bool live = idx < per_phase;
  const float* s = g.slab + (size_t)phase * g.splits * MN + (live ? idx : 0);  // idx = m N + n
  float acc = 0.f;
  if (live) {
    int sp = l;
    for (; sp + 3 * REDW_LANES < g.splits; sp += 4 * REDW_LANES) {
      float t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = s[(size_t)(sp + u * REDW_LANES) * MN];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += t[u];
    }
    for (; sp < g.splits; sp += REDW_LANES) acc += s[(size_t)sp * MN];
  }
  sh[l][ob] = acc;
  __syncthreads();
  for (int h = REDW_LANES / 2; h > 0; h >>= 1) {
    if (l < h) sh[l][ob] += sh[l + h][ob];
    __syncthreads();
  }
  if (l == 0 && live) {
    const uint32_t m = fdiv.div(idx);  // fdiv = N
    const int n = (int)(idx - m * fdiv.d);
    const float wsc = g.wscale ? g.wscale[0] : 1.f;
    const long long ooff = row_offset(g.out, (int)m, MODE == MODE_CONVT2 ? phase : 0) + col_offset(g.out, n);
    float* dst = g.C + ooff;
    float o = red_epi(g, sh[0][ob], wsc, n);
    if (MODE != MODE_WGRAD && g.pmode == 1) o *= act_grad_from_out(g.px[ooff], g.pact, g.palpha);
    *dst = g.accum ? *dst + o : o;
  }
}

// Split-K reduce of a BatchNorm layer's conv forward with the batch statistics fused in:
// the same rows the RED_VEC reduce writes (same split order, bitwise the same values), plus
// the (sum y, sum y^2) of every 64-row segment of every channel in double -- the layout the
// unsplit vector epilogue writes (bnp[(seg * 2 + {0,1}) * N + n], seg = phase * (M / 64) +
// m / 64), so one segment merge serves both and the separate moments pass over y (4 B/elem
// + a launch) is gone.  Block = one 64-row segment x 4*qb columns, thread (rl, q) reduces
// rows rl and rl + RL (RL = 256 / qb) of quad q -- both rows' split loads in flight together,
// as many threads as the plain reduce -- then the per-thread double sums are added over rl
// by a fixed LDS tree (deterministic).  grid = (segments * column chunks, phases).
constexpr int REDBN_QB = 8;

// BWD (pmode 2, the producer's BatchNorm backward sums -- see GemmArgs::pmode): the rows
// written are g = v * act'(y al + be) and the segment sums are (sum g, sum g (y - mean)),
// y read at the rows' own offsets; the same block / tree structure.
template <bool BWD>
__global__ __launch_bounds__(256) void splitk_reduce_bn(GemmArgs g, int mode_t2, int qb) {
  __shared__ double sh[2][256][4];
  const int phase = blockIdx.y;
  const int Q = g.N >> 2, chunks = (Q + qb - 1) / qb;
  const int segm = blockIdx.x / chunks, chunk = blockIdx.x - segm * chunks;
  const int tid = threadIdx.x, lq = tid % qb, q = chunk * qb + lq, rl = tid / qb, RL = 256 / qb;
  const size_t MN = (size_t)g.M * g.N;
  const float* base = g.slab + (size_t)phase * g.splits * MN;
  const float wsc = g.wscale ? g.wscale[0] : 1.f;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (q < Q) {
    const int n = 4 * q;
    const long long noff = col_offset(g.out, n);
    float p_al[4], p_be[4], p_mu[4];
    if constexpr (BWD) {
      const int k = post_seg(g, segm * 64);
#pragma unroll
      for (int i = 0; i < 4; ++i) post_consts(g, k, n + i, p_al[i], p_be[i], p_mu[i]);
    }
    for (int r0 = rl; r0 < 64; r0 += 2 * RL) {  // RL <= 32: two rows per pass
      const int m0 = segm * 64 + r0, m1 = m0 + RL;
      const float* p0 = base + (size_t)m0 * g.N + n;
      const float* p1 = base + (size_t)m1 * g.N + n;
      float4 v0 = *reinterpret_cast<const float4*>(p0), v1 = *reinterpret_cast<const float4*>(p1);
      int sp = 1;
      for (; sp + 4 <= g.splits; sp += 4) {  // split order, as red_sum: 8 loads in flight, then the adds
        float4 a0[4], a1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a0[u] = *reinterpret_cast<const float4*>(p0 + (size_t)(sp + u) * MN);
          a1[u] = *reinterpret_cast<const float4*>(p1 + (size_t)(sp + u) * MN);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v0.x += a0[u].x; v0.y += a0[u].y; v0.z += a0[u].z; v0.w += a0[u].w;
          v1.x += a1[u].x; v1.y += a1[u].y; v1.z += a1[u].z; v1.w += a1[u].w;
        }
      }
      for (; sp < g.splits; ++sp) {
        const float4 a0 = *reinterpret_cast<const float4*>(p0 + (size_t)sp * MN);
        const float4 a1 = *reinterpret_cast<const float4*>(p1 + (size_t)sp * MN);
        v0.x += a0.x; v0.y += a0.y; v0.z += a0.z; v0.w += a0.w;
        v1.x += a1.x; v1.y += a1.y; v1.z += a1.z; v1.w += a1.w;
      }
      const float4 o0 = make_float4(red_epi(g, v0.x, wsc, n), red_epi(g, v0.y, wsc, n + 1),
                                    red_epi(g, v0.z, wsc, n + 2), red_epi(g, v0.w, wsc, n + 3));
      const float4 o1 = make_float4(red_epi(g, v1.x, wsc, n), red_epi(g, v1.y, wsc, n + 1),
                                    red_epi(g, v1.z, wsc, n + 2), red_epi(g, v1.w, wsc, n + 3));
      const long long off0 = row_offset(g.out, m0, mode_t2 ? phase : 0) + noff;
      const long long off1 = row_offset(g.out, m1, mode_t2 ? phase : 0) + noff;
      float a[2][4] = {{o0.x, o0.y, o0.z, o0.w}, {o1.x, o1.y, o1.z, o1.w}};
      if constexpr (BWD) {
        const float4 y0 = *reinterpret_cast<const float4*>(g.px + off0);
        const float4 y1 = *reinterpret_cast<const float4*>(g.px + off1);
        const float yy[2][4] = {{y0.x, y0.y, y0.z, y0.w}, {y1.x, y1.y, y1.z, y1.w}};
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            a[h][i] *= act_grad_from_in(yy[h][i] * p_al[i] + p_be[i], g.pact, g.palpha);
            s1[i] += (double)a[h][i];
            s2[i] += (double)a[h][i] * (double)(yy[h][i] - p_mu[i]);
          }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const double d = (double)a[h][i];
            s1[i] += d;
            s2[i] += d * d;
          }
      }
      *reinterpret_cast<float4*>(g.C + off0) = make_float4(a[0][0], a[0][1], a[0][2], a[0][3]);
      *reinterpret_cast<float4*>(g.C + off1) = make_float4(a[1][0], a[1][1], a[1][2], a[1][3]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) { sh[0][tid][i] = s1[i]; sh[1][tid][i] = s2[i]; }
  __syncthreads();
  for (int h = RL / 2; h > 0; h >>= 1) {  // tid = rl * qb + lq: partner rl + h
    if (rl < h) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sh[0][tid][i] += sh[0][tid + h * qb][i];
        sh[1][tid][i] += sh[1][tid + h * qb][i];
      }
    }
    __syncthreads();
  }
  if (rl == 0 && q < Q) {
    const size_t seg = (size_t)phase * (uint32_t)(g.M >> 6) + (uint32_t)segm;
    double* out = BWD ? g.ppart : g.bnp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[(seg * 2) * g.N + 4 * q + i] = sh[0][tid][i];
      out[(seg * 2 + 1) * g.N + 4 * q + i] = sh[1][tid][i];
    }
  }
}

// ---------------------------------------------------------------- one-output dense layer
// D's closing Conv2d(C, 1, k, 1, 0) over a k x k map (GLI:455, GLI:306) covers the whole
// map: per sample a dot product of C*k*k inputs with the single filter.  As an implicit GEMM
// it is N = 1 (one 32-wide tile column, 1/32 used, split-K 256 ways); here:
//   fwd   one block per sample, y[b] = act(wsc * <x[b], W> + bias)  (fixed-order block sum)
//   dgrad dx[b][e] = (dy[b] * W[e]) * wsc                            (elementwise, NHWC stores)
//   wgrad dW[e] = sum_b dy[b] * x[b][e], b in order                  (thread per filter tap)
// e runs over (h, w, c) with c fastest, so NHWC activations are read/written coalesced; fwd
// and dgrad read the filter packed in the same order (the conv forward pack, [1][(kh,kw,ci)]),
// wgrad writes it in torch order c*k*k + h*k + w.
struct DenseArgs {
  const float* x;             // fwd/wgrad: input.  dgrad: unused
  long long xsb, xsc, xsh, xsw;
  const float* w;
  const float* wscale;
  const float* bias;
  float* y;                   // fwd: output [b * ysb].  dgrad/wgrad: dy (read)
  long long ysb;
  float* out;                 // dgrad: dx (strides xs*).  wgrad: dW (torch layout)
  int B, C, HW, E;            // E = C * HW
  FastDiv fc, fw;             // e -> (hw, c); hw -> (h, w)
  int act;
  float alpha;
  int vec;
  int accum;                  // wgrad: add into out
};

__device__ __forceinline__ long long dense_x_off(const DenseArgs& a, int e, int& widx) {
  const uint32_t hw = a.fc.div(e);
  const int c = e - (int)(hw * a.fc.d);
  const uint32_t h = a.fw.div(hw);
  const int w = (int)(hw - h * a.fw.d);
  widx = c * a.HW + (int)hw;
  return (long long)c * a.xsc + (long long)h * a.xsh + (long long)w * a.xsw;
}

// VEC (host-checked: channel stride 1, C % 4 == 0, 16-B aligned rows): thread items are
// channel quads, one float4 of activations + 4 filter taps.
// VEC (host-checked: channel stride 1, C % 4 == 0, 16-B aligned rows): thread items are
// channel quads, one float4 of activations and one of packed filter.
template <bool VEC>
__global__ __launch_bounds__(1024) void dense1_fwd(DenseArgs a) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const float* xb = a.x + (long long)b * a.xsb;
  float acc = 0.f;
  if constexpr (VEC) {
#pragma unroll 8
    for (int e = 4 * threadIdx.x; e < a.E; e += 4 * 1024) {
      int wi;
      const float4 xv = *reinterpret_cast<const float4*>(xb + dense_x_off(a, e, wi));
      const float4 wv = *reinterpret_cast<const float4*>(a.w + e);
      acc = fmaf(xv.x, wv.x, acc);
      acc = fmaf(xv.y, wv.y, acc);
      acc = fmaf(xv.z, wv.z, acc);
      acc = fmaf(xv.w, wv.w, acc);
    }
  } else {
#pragma unroll 8
    for (int e = threadIdx.x; e < a.E; e += 1024) {
      int wi;
      const long long xo = dense_x_off(a, e, wi);
      acc = fmaf(xb[xo], a.w[e], acc);
    }
  }
  const float t = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const float wsc = a.wscale ? a.wscale[0] : 1.f;
    const float v = t * wsc + (a.bias ? a.bias[0] : 0.f);
    a.y[(long long)b * a.ysb] = act_fwd(v, a.act, a.alpha);
  }
}

// fe = E / (VEC ? 4 : 1): item -> (b, e)
template <bool VEC>
__global__ __launch_bounds__(256) void dense1_dgrad(DenseArgs a, FastDiv fe) {
  const uint32_t total = (uint32_t)a.B * fe.d;
  const float wsc = a.wscale ? a.wscale[0] : 1.f;
  for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < total; idx += gridDim.x * 256u) {
    const uint32_t b = fe.div(idx);
    const int e = (int)(idx - b * fe.d) * (VEC ? 4 : 1);
    int wi;
    const long long xo = dense_x_off(a, e, wi);
    const float g = a.y[(long long)b * a.ysb];
    float* o = a.out + (long long)b * a.xsb + xo;
    if constexpr (VEC) {
      const float4 wv = *reinterpret_cast<const float4*>(a.w + e);
      *reinterpret_cast<float4*>(o) = make_float4((g * wv.x) * wsc, (g * wv.y) * wsc, (g * wv.z) * wsc,
                                                  (g * wv.w) * wsc);
    } else {
      *o = (g * a.w[e]) * wsc;
    }
  }
}

__global__ __launch_bounds__(256) void dense1_wgrad(DenseArgs a) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.E) return;
  int wi;
  const long long xo = dense_x_off(a, e, wi);
  float acc = 0.f;
#pragma unroll 16
  for (int b = 0; b < a.B; ++b) acc = fmaf(a.y[(long long)b * a.ysb], a.x[(long long)b * a.xsb + xo], acc);
  a.out[wi] = a.accum ? a.out[wi] + acc : acc;
}

// WGRAD with 4x4 taps: the GEMM writes C[co][(tap, ci)] with whole-row float4 stores
// (tap-major staging) and this pass turns it into torch layout dW[co][ci][tap].  Writing
// torch layout from the GEMM directly scatters 4-B stores at a 64-B stride (a tile covers
// one tap); on the deep layers (N = 16 Cin up to 16384) that cost ~20 % of the GEMM.
// 16 taps x 64 channels per block through LDS; reads 256-B rows, writes 4 KiB runs.
constexpr int TT_LD = 68;  // (16 t + ci) distinct mod 64 on the read side
__global__ __launch_bounds__(256) void taps_transpose(const float* __restrict__ T, float* __restrict__ O, int Cin,
                                                      long long osb, int accum) {
  __shared__ float sh[16 * TT_LD];
  const int co = blockIdx.y, c0 = blockIdx.x * 64;
  const float* src = T + (size_t)co * 16 * Cin;
  {
    const int t = threadIdx.x >> 4, q = threadIdx.x & 15, c = c0 + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < Cin) v = *reinterpret_cast<const float4*>(src + (size_t)t * Cin + c);
    sh[t * TT_LD + 4 * q] = v.x; sh[t * TT_LD + 4 * q + 1] = v.y;
    sh[t * TT_LD + 4 * q + 2] = v.z; sh[t * TT_LD + 4 * q + 3] = v.w;
  }
  __syncthreads();
  const int ci = threadIdx.x >> 2, tq = threadIdx.x & 3;
  if (c0 + ci < Cin) {
    float4* dst = reinterpret_cast<float4*>(O + (long long)co * osb + (long long)(c0 + ci) * 16 + 4 * tq);
    float4 v = make_float4(sh[(4 * tq) * TT_LD + ci], sh[(4 * tq + 1) * TT_LD + ci], sh[(4 * tq + 2) * TT_LD + ci],
                           sh[(4 * tq + 3) * TT_LD + ci]);
    if (accum) {
      const float4 o = *dst;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    *dst = v;
  }
}

// ---------------------------------------------------------------- weight packing
struct PackArgs {
  const float* W;
  float* out;
  int K, N, phases;
  FastDiv fpci, fpkw;      // k -> (kh, kw, ci)
  FastDiv fnco, fnkw;      // n -> (nh, nw, co)
  long long s_in, s_out, s_kh, s_kw;
  int KH, KW, flip, convt2;
};

// out[phase][n][k] (k contiguous: the GEMM B operand's rows): threads over k, one block
// column per n (n-decomposition uniform per block)
__global__ __launch_bounds__(256) void pack_weights(PackArgs a) {
  const int phase = blockIdx.z;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= a.K) return;
  for (int n = blockIdx.y; n < a.N; n += gridDim.y) {
    uint32_t tn = a.fnco.div(n);
    const int co = n - tn * a.fnco.d;
    uint32_t nh = a.fnkw.div(tn);
    const int nw = tn - nh * a.fnkw.d;
    uint32_t t = a.fpci.div(k);
    const int ci = k - t * a.fpci.d;
    int kh, kw, c_out;
    if (a.convt2) {
      kh = 2 * (int)(t >> 1) + 1 - (phase >> 1);
      kw = 2 * (int)(t & 1) + 1 - (phase & 1);
      c_out = n;
    } else {
      uint32_t kkh = a.fpkw.div(t);
      kh = (int)kkh + (int)nh;
      kw = (int)(t - kkh * a.fpkw.d) + nw;
      c_out = co;
      if (a.flip) {
        kh = a.KH - 1 - kh;
        kw = a.KW - 1 - kw;
      }
    }
    a.out[((size_t)phase * a.N + n) * a.K + k] =
        a.W[ci * a.s_in + c_out * a.s_out + kh * a.s_kh + kw * a.s_kw];
  }
}

// G's 1x1 -> KH x KW first layer (a plain GEMM over z): W[ci][co][tap] contiguous ->
// out[tap * Cout + co][ci] -- a 2-D transpose of [K][N] with the (co, tap) -> (tap, co)
// column permutation.  pack_weights reads that layout a float per 128-B line (one column
// of a K x N matrix per block); here a block moves a 32 (ci) x 128 (co, tap) brick through
// LDS, loaded as float4 rows, stored as 128-B ci runs.
constexpr int PT_K = 32, PT_N = 128;
__global__ __launch_bounds__(256) void pack_t2d(PackArgs a) {
  __shared__ float t[PT_K][PT_N + 1];
  const int T = a.KH * a.KW, Cout = (int)a.fnco.d;
  const int k0 = blockIdx.y * PT_K, j0 = blockIdx.x * PT_N;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 5) + 8 * i, c = 4 * (tid & 31);
    const float4 v = *reinterpret_cast<const float4*>(a.W + (size_t)(k0 + r) * a.N + j0 + c);
    t[r][c] = v.x; t[r][c + 1] = v.y; t[r][c + 2] = v.z; t[r][c + 3] = v.w;
  }
  __syncthreads();
  const int jl = tid >> 1, h = tid & 1, j = j0 + jl;
  const int co = j / T, tap = j - co * T;
  float* dst = a.out + (size_t)(tap * Cout + co) * a.K + k0 + 16 * h;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(dst + 4 * q) = make_float4(t[16 * h + 4 * q][jl], t[16 * h + 4 * q + 1][jl],
                                                          t[16 * h + 4 * q + 2][jl], t[16 * h + 4 * q + 3][jl]);
}

// ---------------------------------------------------------------- narrow convolutions
// The image layers do not fit the pipelined GEMM: N <= 4 wastes >= 88% of a 32-wide MFMA
// tile, and K = 16*CI <= 64 is one or two BK tiles around a full prologue and epilogue:
//   convt2_narrow_mfma   k4 s2 p1 ConvTranspose2d (and the Conv2d dgrad of the same shape)
//                        with <= 4 output channels: G's image layer (GLI:448) and D's image
//                        gradient (the backward of GLI:410 into G), on 4x4x1 MFMA blocks.
//   conv_narrow_in_mfma  Conv2d with <= 4 input channels and a 4x4 kernel: D's image layer
//                        (GLI:410) as a single-pass MFMA tile (below).
struct NarrowArgs {
  const float* x;
  long long xsb, xsc, xsh, xsw;
  int B, H, W, C;         // input grid
  const float* w;         // NARROW_T: packed [C][4][64] (pack_narrow);  NARROW_IN: torch [Cout][C][KH][KW]
  float* y;
  long long ysb, ysc, ysh, ysw;
  int Ho, Wo, Cout;
  int stride, pad;
  const float* bias;
  const float* wscale;
  int act;
  float alpha;
  int x_bytes, y_bytes;   // conv_img_in: byte extents of x and y (< 2^31, buffer descriptors)
  int splits = 1, cps = 0;  // convt2_narrow_mfma: input-channel splits (cps channels each, a multiple of 16)
  float* slab = nullptr;  // ... their raw sums [split][b][co][oh][ow] when splits > 1 (narrow_split_reduce)
  // conv3_narrow_out: weight element (out n, in c, tap t) at
  // w[n * w_sn + c * w_sc + (w_flip ? taps - 1 - t : t)] (torch Conv2d layout: w_sn = C * taps,
  // w_sc = taps; a data gradient reads the kernel transposed and flipped)
  long long w_sn = 0, w_sc = 0;
  int w_flip = 0;
  // wgrad3_narrow: dy (the layer's output gradient) and its strides; blocks of `rows` output rows
  const float* dy = nullptr;
  long long dsb = 0, dsc = 0, dsh = 0, dsw = 0;
  int chunks = 0, rows = 0;
};

// Conv2d with a 4x4 kernel and CI <= 4 input channels (D's image layer, GLI:410) as ONE MFMA
// GEMM tile pass: M = output pixels, N = Cout, K = 16*CI (16..64).  K is too short for the
// pipelined GEMM (one or two BK tiles around a full prologue/epilogue, and a per-element
// im2col index decomposition in every tile), so a block builds its whole 128 x K im2col
// tile once (per-row pixel decomposition, per-k (ci, kh, kw) from bit fields), stages the
// 128 x K weight tile straight from torch layout ([co][ci][kh][kw] = [n][k], k-contiguous),
// and runs K/2 MFMA steps per accumulator from k-contiguous LDS rows (row stride K+4 dwords,
// an odd number of 16-B slots: conflict-free ds_read_b128; lane half h takes k in
// [h K/2, (h+1) K/2)).  Persistent over M tiles (next tile's im2col loads in flight during
// this tile's MFMAs); the product is formed transposed (rows = channels) so the NHWC
// epilogue is one float4 store per 4 channels.  Measured (C2 D image layer, 64x3x128^2 ->
// 128 ch): 100 us as one VALU thread per pixel, 76 us here; without the stores 53 us --
// fp32 MFMA and VALU share one issue pipe on gfx950, so the im2col/epilogue VALU is paid
// in MFMA time.
template <int CI>
__global__ __launch_bounds__(256, 2) void conv_narrow_in_mfma(NarrowArgs a) {
  constexpr int K = CI * 16, KH2 = K / 2, LD = K + 4;
  __shared__ __attribute__((aligned(16))) float As[128 * LD];
  __shared__ __attribute__((aligned(16))) float Bs[128 * LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, lk = lane >> 5;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  __shared__ long long moff[128];
  const int HWo = a.Ho * a.Wo, M = a.B * HWo, tiles = (M + 127) / 128;
  const int n0 = blockIdx.y * 128;
  {
    // all K/2 weight loads in flight before the first LDS store (a rolled loop would wait
    // on each load in turn: ~24 serialised L2 round trips per block)
    float wv[K / 2];
#pragma unroll
    for (int j = 0; j < K / 2; ++j) {
      const int e = tid + 256 * j, r = e / K, k = e - r * K, n = n0 + r;
      wv[j] = n < a.Cout ? a.w[(size_t)n * K + k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < K / 2; ++j) {
      const int e = tid + 256 * j, r = e / K, k = e - r * K;
      Bs[r * LD + k] = wv[j];
    }
  }
  // im2col of one tile into registers: thread = (row tid/2, half tid%2 of the K columns)
  const int row = tid >> 1, half = tid & 1;
  float av[KH2];
  auto gather = [&](int m0) {
    const int m = m0 + row;
    if (m < M) {
      const int b = m / HWo, rem = m - b * HWo, oi = rem / a.Wo, oj = rem - oi * a.Wo;
      const int ih0 = oi * a.stride - a.pad, iw0 = oj * a.stride - a.pad;
      const float* xb = a.x + (long long)b * a.xsb;
#pragma unroll
      for (int kk = 0; kk < KH2; ++kk) {
        const int k = half * KH2 + kk, ci = k >> 4, ih = ih0 + ((k >> 2) & 3), iw = iw0 + (k & 3);
        av[kk] = ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                     ? xb[(long long)ci * a.xsc + (long long)ih * a.xsh + (long long)iw * a.xsw]
                     : 0.f;
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KH2; ++kk) av[kk] = 0.f;
    }
  };
  const float wsc = a.wscale ? a.wscale[0] : 1.f;
  const float* Ar = As + (wm + l32) * LD + lk * KH2;
  const float* Br = Bs + (wn + l32) * LD + lk * KH2;
  // persistent over M tiles: the next tile's im2col loads are in flight during this tile's
  // MFMAs and stores (one block per tile spent most of its life waiting on them)
  int t = blockIdx.x;
  if (t < tiles) gather(t * 128);
  for (; t < tiles; t += gridDim.x) {
    const int m0 = t * 128;
#pragma unroll
    for (int kk = 0; kk < KH2; ++kk) As[row * LD + half * KH2 + kk] = av[kk];
    if (tid < 128) {
      const int m = m0 + tid;
      long long o = -1;
      if (m < M) {
        const int b = m / HWo, rem = m - b * HWo, oi = rem / a.Wo, oj = rem - oi * a.Wo;
        o = (long long)b * a.ysb + (long long)oi * a.ysh + (long long)oj * a.ysw;
      }
      moff[tid] = o;
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) gather((t + gridDim.x) * 128);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // transposed product: rows = output channels (A = weights), columns = pixels (B =
    // im2col), so each lane holds 4 consecutive channels of one pixel per register quad
    // and the NHWC store is one float4
#pragma unroll
    for (int q = 0; q < KH2 / 4; ++q) {
      float4 a4[2], b4[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        a4[u] = *reinterpret_cast<const float4*>(Ar + 32 * u * LD + 4 * q);
        b4[u] = *reinterpret_cast<const float4*>(Br + 32 * u * LD + 4 * q);
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(b4[j][s4], a4[i][s4], acc[i][j], 0, 0, 0);
    }
    const bool vec4 = a.ysc == 1 && (a.Cout & 3) == 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long long o = moff[wm + 32 * i + l32];  // this lane's pixel
      if (o < 0) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int cb = n0 + wn + 32 * j + 8 * g + 4 * lk;  // channels cb .. cb+3
          if (cb >= a.Cout) continue;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = act_fwd(acc[i][j][4 * g + e] * wsc + (a.bias && cb + e < a.Cout ? a.bias[cb + e] : 0.f), a.act,
                           a.alpha);
          if (vec4) {
            *reinterpret_cast<float4*>(a.y + o + cb) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (cb + e < a.Cout) a.y[o + (long long)(cb + e) * a.ysc] = v[e];
          }
        }
    }
    __syncthreads();  // As / moff are rewritten for the next tile
  }
}

// Conv2d 3x3 stride 1 with NC <= 4 output channels over an NHWC input of C channels (C a power
// of two, 4 <= C <= 256): arch 1's image layer (GLI:222-223) and, reading the kernel transposed
// and flipped, the data gradient of arch 1's 3-channel input layer (GLI:202, the WGAN-GP input
// gradient).  As an implicit GEMM (N = NC) every MFMA would be >= 7/8 padding.  Here L = C / 4
// lanes share a pixel, lane l owning channels 4 l .. 4 l + 3: it holds their 9 x 4 x NC weights
// in registers for the whole wave, so a pixel costs each lane 9 float4 loads (the L lanes of a
// tap read one contiguous C * 4-byte run) and 36 NC FMAs, after which a log2(L)-step xor
// butterfly adds the lanes (a + b == b + a: every lane of a pixel holds the same sums) and lane
// o mod L stores output o.  A wave walks `steps` groups of 64 / L pixels, two groups' loads in
// flight together; waves are independent (no LDS, no barrier).  Round 6: a thread
// per (pixel, quarter of the channels) ran 9 x C / 16 dependent load -> FMA steps at C4 (C =
// 128), latency-bound at 14.1 us per call whatever the pixels per thread.
constexpr int N3_MAXC = 256;
constexpr int N3_WAVES = 4;  // waves per block
template <int NC>
__global__ __launch_bounds__(64 * N3_WAVES) void conv3_narrow_out(NarrowArgs a, int steps) {
  extern __shared__ float wl[];  // [L][9][4][NC]: lane sl's weights contiguous
  const int C = a.C, L = C >> 2, PW = 64 / L;
  const int lc = __builtin_ctz(C);  // C is a power of two
  for (int i = threadIdx.x; i < 9 * C * NC; i += 64 * N3_WAVES) {
    const int o = i % NC, e = i / NC, c = e & (C - 1), t = e >> lc;  // reads: o fastest, then channel
    wl[(((c >> 2) * 9 + t) * 4 + (c & 3)) * NC + o] =
        a.w[o * (int)a.w_sn + c * (int)a.w_sc + (a.w_flip ? 8 - t : t)];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, sl = lane & (L - 1);
  const int HW = a.Ho * a.Wo, P = a.B * HW;  // < 2^31 (plan)
  const int pix0 = (blockIdx.x * N3_WAVES + (threadIdx.x >> 6)) * steps * PW;
  if (pix0 >= P) return;  // whole wave: no barrier below
  float w[9][4][NC];
  {
    const float* src = wl + sl * 36 * NC;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int o = 0; o < NC; ++o) w[t][k][o] = src[(t * 4 + k) * NC + o];
  }
  const float wsc = a.wscale ? a.wscale[0] : 1.f;
  float bo[NC];
#pragma unroll
  for (int o = 0; o < NC; ++o) bo[o] = a.bias ? a.bias[o] : 0.f;
  // x through a buffer descriptor: a tap outside the image (or a pixel past P) gets an offset
  // past the extent and the load returns zeros -- every load unconditional, no branch (a
  // conditional load is compiled into a branch that waits for it: one load in flight)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const int xsb = 4 * (int)a.xsb, xsh = 4 * (int)a.xsh, xsw = 4 * (int)a.xsw;  // bytes
  // the lane's pixel (b, oh, ow), advanced by PW per group without a division
  int pix = pix0 + lane / L, b = pix / HW, r = pix - b * HW, oh = r / a.Wo, ow = r - oh * a.Wo;
  auto advance = [&]() {
    pix += PW;
    ow += PW;
    while (ow >= a.Wo) {
      ow -= a.Wo;
      if (++oh == a.Ho) { oh = 0; ++b; }
    }
  };
  auto load = [&](u32x4 (&xv)[9]) {
    const int base = b * xsb + (oh - a.pad) * xsh + (ow - a.pad) * xsw + 16 * sl;
    const bool in = pix < P;
    bool rok[3], cok[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      rok[k] = in & ((unsigned)(oh + k - a.pad) < (unsigned)a.H);
      cok[k] = (unsigned)(ow + k - a.pad) < (unsigned)a.W;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t)
      xv[t] = __builtin_amdgcn_raw_buffer_load_b128(
          xr, (rok[t / 3] & cok[t % 3]) ? base + (t / 3) * xsh + (t % 3) * xsw : 0x7ffffff0, 0, 0);
  };
  auto finish = [&](const u32x4 (&xv)[9], int pb, int ob, int ohb, int owb) {
    float acc[NC];
#pragma unroll
    for (int o = 0; o < NC; ++o) acc[o] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float x0 = __uint_as_float(xv[t].x), x1 = __uint_as_float(xv[t].y), x2 = __uint_as_float(xv[t].z),
                  x3 = __uint_as_float(xv[t].w);
#pragma unroll
      for (int o = 0; o < NC; ++o) acc[o] += x0 * w[t][0][o] + x1 * w[t][1][o] + x2 * w[t][2][o] + x3 * w[t][3][o];
    }
    for (int m = 1; m < L; m <<= 1)
#pragma unroll
      for (int o = 0; o < NC; ++o) acc[o] += __shfl_xor(acc[o], m);
    if (pb >= P) return;
    float* yp = a.y + ob * a.ysb + (long long)ohb * a.ysh + (long long)owb * a.ysw;
    if (L >= NC) {  // lane o stores output o: one activation per lane
      if (sl < NC) {
        float v = acc[0], bb = bo[0];
#pragma unroll
        for (int o = 1; o < NC; ++o) {
          v = sl == o ? acc[o] : v;
          bb = sl == o ? bo[o] : bb;
        }
        yp[(long long)sl * a.ysc] = act_fwd(v * wsc + bb, a.act, a.alpha);
      }
    } else {
#pragma unroll
      for (int o = 0; o < NC; ++o)
        if ((o & (L - 1)) == sl) yp[(long long)o * a.ysc] = act_fwd(acc[o] * wsc + bo[o], a.act, a.alpha);
    }
  };
  // two pixel groups per pass: 18 loads in flight, the first group's FMAs waiting only on its own
  for (int st = 0; st < steps; st += 2) {
    u32x4 xa[9], xb[9];
    load(xa);
    const int pa = pix, ba = b, oha = oh, owa = ow;
    advance();
    if (st + 1 >= steps) pix = P;  // odd tail: the second group is empty
    load(xb);
    const int pb = pix, bb = b, ohb = oh, owb = ow;
    advance();
    finish(xa, pa, ba, oha, owa);
    finish(xb, pb, bb, ohb, owb);
  }
}

// Weight gradient of a 3x3 stride-1 pad-1 Conv2d with NC <= 4 output channels over a CW-channel
// input (CW % 4 == 0; arch 1's 3-channel output layer, GLI:222): dW[co][ci][kh][kw] = sum_p
// dy[p][co] x[p + (kh, kw) - 1][ci].  A block owns R whole output rows of one image (R * Wo <=
// N3W_PIX): it first stages their dy rows and the R + 2 x rows around them (zero halo) in LDS
// with every thread's loads in flight together, then thread (tap, 4 input channels) accumulates
// its 4 x NC outputs over the block's pixels in order from LDS.  The per-block partials go to a
// slab in the WGRAD GEMM's [split][co][(kh, kw, ci)] layout, which splitk_reduce(_wide) adds in
// block order into torch layout (and into .grad when accumulating).  As a GEMM this is M = NC:
// a 128 x 128 tile >= 97 % padding (88 us per C4 call; here 14.7 us + the reduce).  The
// mirror case (<= 4 input channels, arch 1's input layer) stays on the GEMM: the same staging
// measured 40 us per call against its 29 us (K = 9 NC is only short, M is full).
constexpr int N3W_PIX = 128;
constexpr int N3W_UNR = 8;  // x-halo float4 loads in flight per thread
template <int NC>
__global__ void wgrad3_narrow(NarrowArgs a, int CW, int R) {
  extern __shared__ __attribute__((aligned(16))) float sm3[];
  const int Wo = a.Wo, XW = Wo + 2;
  float* xs = sm3;                          // [(R + 2) * XW][CW]
  float* ds = sm3 + (R + 2) * XW * CW;      // [R * Wo][NC]
  const int rows_per_img = (a.Ho + R - 1) / R, b = blockIdx.x / rows_per_img;
  const int oh0 = (blockIdx.x - b * rows_per_img) * R, nr = min(R, a.Ho - oh0);
  const int tid = threadIdx.x, nt = blockDim.x;
  // stage: x rows oh0 - 1 .. oh0 + nr (zero outside the image), dy rows oh0 .. oh0 + nr - 1
  const int xn = (R + 2) * XW * CW;
  if (a.xsc == 1 && ((a.xsw | a.xsh | a.xsb) & 3) == 0 && ((uintptr_t)a.x & 15) == 0) {
    // NHWC: float4 per (pixel, 4 channels), N3W_UNR loads in flight per thread before the LDS
    // stores (round 6: the scalar loop below kept ~1 load in flight -- 33.6 us per C4 call)
    const int CQ = CW / 4, xq = xn / 4;
    for (int i0 = tid; i0 < xq; i0 += N3W_UNR * nt) {
      float4 v[N3W_UNR];
#pragma unroll
      for (int u = 0; u < N3W_UNR; ++u) {
        const int i = i0 + u * nt;
        const int cq = i % CQ, pix = i / CQ, rr = pix / XW, cc = pix - rr * XW;
        const int ih = oh0 - 1 + rr, iw = cc - 1;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < xq && rr < nr + 2 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
          v[u] = *reinterpret_cast<const float4*>(a.x + (long long)b * a.xsb + (long long)ih * a.xsh +
                                                  (long long)iw * a.xsw + 4 * cq);
      }
#pragma unroll
      for (int u = 0; u < N3W_UNR; ++u)
        if (i0 + u * nt < xq) reinterpret_cast<float4*>(xs)[i0 + u * nt] = v[u];
    }
  } else {
    for (int i = tid; i < xn; i += nt) {
      const int c = i % CW, pix = i / CW, rr = pix / XW, cc = pix - rr * XW;
      const int ih = oh0 - 1 + rr, iw = cc - 1;
      xs[i] = (rr < nr + 2 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                  ? a.x[(long long)b * a.xsb + (long long)c * a.xsc + (long long)ih * a.xsh + (long long)iw * a.xsw]
                  : 0.f;
    }
  }
  const int dn = nr * Wo * NC;
  for (int i = tid; i < dn; i += nt) {
    const int c = i % NC, pix = i / NC, rr = pix / Wo, cc = pix - rr * Wo;
    ds[i] = a.dy[(long long)b * a.dsb + (long long)c * a.dsc + (long long)(oh0 + rr) * a.dsh + (long long)cc * a.dsw];
  }
  __syncthreads();
  const int q = tid % (CW / 4), t = tid / (CW / 4);
  if (t >= 9) return;
  const int kh = t / 3, kw = t % 3;
  float acc[4][NC];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[e][c] = 0.f;
  for (int rr = 0; rr < nr; ++rr) {
    const float* xr = xs + ((rr + kh) * XW + kw) * CW + 4 * q;
    const float* dr = ds + rr * Wo * NC;
    for (int cc = 0; cc < Wo; ++cc) {
      const float4 xv = *reinterpret_cast<const float4*>(xr + cc * CW);
      const float x4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[e][c] += x4[e] * dr[cc * NC + c];
    }
  }
  // slab [block][co][(t, ci)]: M = NC rows of N = 9 CW
  float* sl = a.slab + (size_t)blockIdx.x * NC * 9 * CW;
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int c = 0; c < NC; ++c) sl[((size_t)c * 9 + t) * CW + 4 * q + e] = acc[e][c];
}

// bytes of wgrad3_narrow's LDS staging for R output rows
static inline size_t wgrad3_lds_bytes(int R, int Wo, int CW, int NC) {
  return (size_t)((R + 2) * (Wo + 2) * CW + R * Wo * NC) * 4;
}

// Conv2d k4 s2 p1 over an image with CI <= 3 channels producing Cout % 128 == 0 channels
// NHWC (D's image layer GLI:410, and G's image-layer data gradient).  K = 16 CI is too
// short for the pipelined GEMM, and the layer both runs 6.4 GFLOP of fp32 MFMA and streams
// a 128-channel output (C3 shard: 268 MB).  Every WAVE is an independent persistent worker
// (no block barrier anywhere in the loop: the per-tile barrier of a block-shared window held
// the MFMA pipe at ~50 % through convoys of waves waiting for each other):
//   * a wave tile is 32 consecutive output pixels (a row segment, or 2 rows of 16) x the
//     block's 128 channels: 4 accumulators of 32 x 32, channels as MFMA rows;
//   * the wave's 128 x K weights (x the spectral 1/sigma) stay in VGPRs, so each MFMA step
//     reads ONE im2col operand from LDS (a ds_read_b32 at a compile-time offset) for 4
//     MFMAs; the bias is the accumulators' initial value;
//   * its input window (2R+2 rows x 2 WS+8 columns x CI, 16-B aligned) arrives by LDS-DMA
//     (buffer_load_dwordx4 ... lds into a wave-private double buffer, one tile ahead); the
//     zero padding is the buffer's out-of-range read (whole float4s lie inside or outside
//     the image: W % 4 == 0);
//   * epilogue per 32-channel group: activation, staging in a wave-private XOR-swizzled LDS
//     tile, read back as 128-B channel runs, buffer stores with SGPR offsets.
// fp32 MFMA and VALU share an issue pipe on gfx950: the VALU left is 2 per activated value
// and 4 per DMA piece; two waves per SIMD hide each other's epilogue behind their MFMAs.
// Measured at the C3 shape (32 x 3 x 256^2 -> 128 ch, tools/narrow_micro.py, HIP events
// incl. a ~6 us launch floor): 133 us for the block-tiled predecessor, 79 us here.  The
// same loop without the epilogue runs at the MFMA roof (~43 us); the prologue's weight
// staging must be bank-conflict free (row stride K + 1: an 8-way conflicted version cost
// 9 us per launch).
typedef int i32x4 __attribute__((ext_vector_type(4)));
// byte address of an LDS location, wave-uniform (M0 operand of an LDS-DMA)
__device__ __forceinline__ int lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane((int)(uintptr_t)(const __attribute__((address_space(3))) float*)p);
}
// One 16-B-per-lane LDS-DMA piece: lane l's 16 bytes at byte offset voff of the raw buffer
// land at LDS byte m0 + 16 l (an out-of-range voff writes zeros).
__device__ __forceinline__ void dma_lds16(int m0, int voff, i32x4 rsrc) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

// One 16-B-per-lane buffer store (raw descriptor rsrc, per-lane voff, wave-uniform soff) followed
// by wait states IN THE SAME STATEMENT, so no instruction can sit between the store and them.
// gfx950 does not interlock a VALU write of a wide store's data VGPRs against the store still
// reading them, and LLVM inserts no wait state for a MUBUF store whose soffset is an SGPR: with
// two blocks per CU a v_mul writing the data's first VGPR right behind the store replaced the
// first dword of lanes 12-15 of every 16 (C2 / C3 image layers: 0.1-1 % of D's first-layer
// outputs wrong on every wave's second and later tiles; tools/img_in_check.py).
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_guarded(float4 f, int voff, i32x4 rsrc, int soff) {
  const f32x4v v = {f.x, f.y, f.z, f.w};
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 4"
               :
               : "v"(v), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory");
}

// NI: 32-channel groups per block (4: 128-channel tiles; 1: 32-channel tiles for narrow D widths)
template <int CI, int WS, int ACT, int NI = 4>  // ACT 0: identity, 1: max(v, v * neg) (ReLU / LeakyReLU, neg <= 1), 2: act_fwd
__global__ __launch_bounds__(256, 2) void conv_img_in(NarrowArgs a, int tiles) {
  constexpr int NCH = 32 * NI;                    // output channels per block
  constexpr int K = CI * 16, NS = K / 2;          // MFMA steps (32x32x2)
  constexpr int RW = 32 / WS;                     // output rows per wave tile (1 or 2)
  constexpr int RR = 2 * RW + 2, CW = 2 * WS + 8; // window rows, columns (image cols 2 oj0 - 4 ..)
  constexpr int WCH = RR * CW;                    // window floats per channel
  constexpr int WIN = CI * WCH, NQ = WIN / 4;     // window floats, float4s
  constexpr int QPL = (NQ + 63) / 64;             // DMA pieces per lane
  constexpr int WSTG = (NCH * (K + 1) + 511) / 512 * 64;  // 1/8 of the prologue's weight staging
  constexpr int WBUF = QPL * 256 > WSTG ? QPL * 256 : WSTG;  // one window buffer (floats)
  constexpr int RD = 4;                           // im2col read-ahead (MFMA steps)
  constexpr int OOB_OFF = 0x7ffffff0;
  static_assert(CW % 4 == 0 && WIN % 4 == 0, "window rows are float4-aligned");
  __shared__ __attribute__((aligned(16))) float win[4][2][WBUF];
  __shared__ __attribute__((aligned(16))) float stg[4][32 * 32];  // per wave [pixel][channel quad ^ swz]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, lk = lane >> 5;
  const int n0 = blockIdx.y * NCH;
  const int HWo = a.Ho * a.Wo;
  // raw buffer descriptor of x for the DMA pieces (stride 0, num_records = byte extent)
  const i32x4 xd = {(int)(uintptr_t)a.x, (int)((uintptr_t)a.x >> 32), a.x_bytes, 0x00020000};
  const i32x4 yd = {(int)(uintptr_t)a.y, (int)((uintptr_t)a.y >> 32), a.y_bytes, 0x00020000};
  // weights: wa[i][s] = W[n0 + 32 i + l32][2 s + lk] / sigma  (torch [Cout][CI][4][4] = [n][k])
  // (staged through LDS by the whole block with coalesced loads: NCH x K floats, once)
  // (every global load of the prologue is issued before the first wait: at ~1-2 us per
  // round trip, a dependent sequence of them costs as much as several tiles)
  constexpr int WLD = (NCH * K + 255) / 256;
  float wtmp[WLD];
#pragma unroll
  for (int q = 0; q < WLD; ++q) {
    const int e = tid + 256 * q;
    wtmp[q] = e < NCH * K ? a.w[(size_t)n0 * K + e] : 0.f;
  }
  const float wsc = a.wscale ? a.wscale[0] : 1.f;
  float wb[NI];  // bias column (see below)
#pragma unroll
  for (int i = 0; i < NI; ++i) wb[i] = (a.bias && lk == 0) ? a.bias[n0 + 32 * i + l32] : 0.f;
  {
    float* wst = &win[0][0][0];  // the window buffers are free until the first DMA
    static_assert(4 * 2 * WBUF >= NCH * (K + 1), "weight staging fits the window buffers");
#pragma unroll
    for (int q = 0; q < WLD; ++q) {
      const int e = tid + 256 * q, r = e / K;  // row stride K + 1: conflict-free reads below
      if (e < NCH * K) wst[e + r] = wtmp[q];
    }
    __syncthreads();
  }
  float wa[NI][NS];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s) wa[i][s] = win[0][0][(32 * i + l32) * (K + 1) + 2 * s + lk];
  if (a.wscale) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int s = 0; s < NS; ++s) wa[i][s] *= wsc;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(wa[i][s]));  // resident: no re-load in the loop
  // bias as one extra MFMA step per accumulator (wb: k0 = bias, k1 = 0, against a column of
  // ones): the accumulators start from it exactly, with no per-tile LDS reads
  const float one_k0 = lk == 0 ? 1.f : 0.f;
  __syncthreads();  // weight staging read before the window buffers are reused
  // this lane's pixel: row pr, column pc of the wave tile; window base of its im2col reads
  const int pr = l32 / WS, pc = l32 - pr * WS;
  const int base = 2 * pr * CW + 2 * pc + 3 + lk;
  // DMA piece q of this lane = window float4 f = 64 q + lane = (c, rr, c4): source byte offset
  // relative to the tile's (2 oi0, 2 oj0) corner, and edge flags (1 left float4, 2 right,
  // 4 top row, 8 bottom row, 16 beyond the window), 5 bits per piece
  int wofs[QPL], wflag = 0;
#pragma unroll
  for (int q = 0; q < QPL; ++q) {
    const int f = 64 * q + lane;
    const int c = f / (WCH / 4), r2 = f - c * (WCH / 4), rr = r2 / (CW / 4), c4 = r2 - rr * (CW / 4);
    wofs[q] = (int)(((long long)c * a.xsc + (long long)(rr - 1) * a.xsh + (long long)(4 * c4 - 4)) * 4);
    const int fl = f >= NQ ? 16 : (c4 == 0 ? 1 : 0) | (c4 == CW / 4 - 1 ? 2 : 0) | (rr == 0 ? 4 : 0) | (rr == RR - 1 ? 8 : 0);
    wflag |= fl << (5 * q);
  }
  auto tile_pos = [&](int t, int& b, int& oi0, int& oj0) {
    const int m0 = t * 32;
    b = m0 / HWo;
    const int rem = m0 - b * HWo;
    oi0 = rem / a.Wo;
    oj0 = rem - oi0 * a.Wo;
  };
  auto fetch = [&](int t, float* dst) {
    int b, oi0, oj0;
    tile_pos(t, b, oi0, oj0);
    const int mask = 16 | (oj0 == 0 ? 1 : 0) | (oj0 + WS >= a.Wo ? 2 : 0) | (oi0 == 0 ? 4 : 0) | (oi0 + RW >= a.Ho ? 8 : 0);
    const int tb = (int)(((long long)b * a.xsb + 2LL * oi0 * a.xsh + 2LL * oj0) * 4);
#pragma unroll
    for (int q = 0; q < QPL; ++q) {
      const int off = ((wflag >> (5 * q)) & mask) ? OOB_OFF : wofs[q] + tb;
      dma_lds16(lds_addr(dst + 256 * q), off, xd);
    }
  };
  // epilogue geometry: staging T[pixel][quad ^ ((pixel >> 1) & 7)] (conflict-free writes of
  // (pixel l32, quad 2g + lk) and reads of (pixel 8u + lane / 8, quad lane % 8)); each store
  // instruction writes 8 pixels x 128 B
  float* T = stg[wid];
  const int rq = lane & 7, rp = lane >> 3;
  const int lvo = (int)(((long long)rp * a.ysw + 4 * rq + n0) * 4);
  const int ysh4 = (int)(a.ysh * 4), ysw4 = (int)(a.ysw * 4);
  const float neg = a.act == RGAN_ACT_RELU ? 0.f : a.alpha;
  auto actf = [&](float v) {
    if constexpr (ACT == 0) return v;
    else if constexpr (ACT == 1) return vmaxf(v, v * neg);
    else return act_fwd(v, a.act, a.alpha);
  };
  const int G = (int)gridDim.x * 4;
  int t = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wid);  // wave-uniform (SGPR)
  if (t >= tiles) return;
  float* W0 = win[wid][0];
  float* W1 = win[wid][1];
  fetch(t, W0);
  // one wave tile: MFMAs from window Wr, then the next tile's window into Wn, then the
  // epilogue.  The DMA pieces are inline asm (dma_lds16), invisible to the compiler's wait
  // insertion -- which cannot tell the buffers apart and would stall every later LDS read on
  // them -- so the waits for them are the explicit vmcnt below, and nothing else in the loop
  // loads from global memory
  auto tile = [&](int t, const float* Wr, float* Wn, auto first_c) {
    const int tn = t + G;
    const bool more = tn < tiles;
    // this tile's window landed: the previous tile's 16 stores went out after its DMA and
    // may stay in flight (vmcnt retires in issue order)
    // (NI x 4 stores per tile: vmcnt(4 NI); a fixed vmcnt(16) let the 32-channel tiles read
    // their window before its DMA landed)
    constexpr int VMC = 4 * NI, VMC_ENC = 0x0f70 | (VMC & 15) | ((VMC >> 4) << 14);
    if constexpr (decltype(first_c)::value) __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    else __builtin_amdgcn_s_waitcnt(VMC_ENC);                                     // vmcnt(4 NI)
    float bv[NS];
    auto read_step = [&](int s) {
      // k = 2 s + lk = 16 ci + 4 kh + kw; the lk part is in base (kw parity)
      const int k0 = 2 * s, ci = k0 >> 4, kh = (k0 >> 2) & 3, kw = k0 & 3;
      bv[s] = Wr[base + ci * WCH + kh * CW + kw];
    };
#pragma unroll
    for (int s = 0; s < RD && s < NS; ++s) read_step(s);
    f32x16 acc[NI];
    const f32x16 zero = {};
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(wb[i], one_k0, zero, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + RD < NS) read_step(s + RD);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[i][s], bv[s], acc[i], 0, 0, 0);
    }
    if (more) fetch(tn, Wn);
    int b, oi0, oj0;
    tile_pos(t, b, oi0, oj0);
    const int tb4 = (int)(((long long)b * a.ysb + (long long)oi0 * a.ysh + (long long)oj0 * a.ysw) * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int quad = 2 * g + lk;
        *reinterpret_cast<float4*>(T + l32 * 32 + 4 * (quad ^ ((l32 >> 1) & 7))) =
            make_float4(actf(acc[i][4 * g]), actf(acc[i][4 * g + 1]), actf(acc[i][4 * g + 2]), actf(acc[i][4 * g + 3]));
      }
      float4 ev[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pl = 8 * u + rp;
        ev[u] = *reinterpret_cast<const float4*>(T + pl * 32 + 4 * (rq ^ ((pl >> 1) & 7)));
      }

#pragma unroll
      for (int u = 0; u < 4; ++u) {
        // pixels 8 u .. 8 u + 7 of the wave tile lie in one output row (WS >= 16); the
        // store carries its own wait states (store16_guarded)
        const int p = 8 * u, prr = p / WS, pcc = p - prr * WS;
        const int so = __builtin_amdgcn_readfirstlane(tb4 + prr * ysh4 + pcc * ysw4 + 128 * i);
        store16_guarded(ev[u], lvo, yd, so);
      }
    }
  };
  using F = std::integral_constant<bool, false>;
  using Tr = std::integral_constant<bool, true>;
  tile(t, W0, W1, Tr{});
  for (;;) {
    t += G;
    if (t >= tiles) break;
    tile(t, W1, W0, F{});
    t += G;
    if (t >= tiles) break;
    tile(t, W0, W1, F{});
  }
}

// k4 s2 p1 ConvTranspose2d with NC <= 4 output channels on v_mfma_f32_4x4x1_16b_f32: 16
// independent 4x4 outer products per instruction, so the 4 output channels fill the N
// dimension (75% useful at NC = 3 against 9% for a 32-wide tile) and the 64 lanes are 64
// input-grid pixels: lane 4b+i supplies pixel 4b+i's input value (A row i of block b),
// lane 4b+j the weight of output channel j (B column j, the same in every block); lane
// 4b+j receives D[b][i][j] = pixel 4b+i, channel j.  Each of the 16 (phase, tap) pairs is
// one K=1 step per input channel: output (2i+ph, 2j+pw) <- input (i+ph-th, j+pw-tw) through
// tap (2th+1-ph, 2tw+1-pw), th, tw in {0, 1}.
// Block: 16 x 32 input pixels (4 waves x 2 groups of 4 x 16), the (18 x 34)-pixel halo
// staged through LDS 16 channels at a time (pixel stride 20 dwords: ds_read_b128 of 4
// channels), weights [co][c][tap] staged beside it; per 4 channels a wave reads 18 + 16
// ds_read_b128 and issues 128 MFMAs.
constexpr int NARROW_MAX_SPLITS = 8;  // input-channel splits of convt2_narrow_mfma on small grids
constexpr int NM_TR = 16, NM_TC = 32, NM_HR = NM_TR + 2, NM_HC = NM_TC + 2, NM_CH = 16, NM_LD = NM_CH + 4;
constexpr int NM_XQ = NM_HR * NM_HC * (NM_CH / 4);  // float4 slots of one staged chunk
// LDS row stride of the staged halo: a multiple of 64 dwords, so that the two image rows a
// ds_read_b128 lane group spans (lanes 0-3 and 12-15 of one row, 20-27 of the next: the
// MI355X_MICROARCH.md LDS table) land on disjoint banks -- at the packed 680-dword stride
// (34 pixels x 20) they overlapped two ways (SQ_LDS_BANK_CONFLICT 11.9M cycles per C3 launch)
constexpr int NM_RS = (NM_HC * NM_LD + 63) / 64 * 64;
constexpr int NM_XPT = (NM_XQ + 255) / 256;         // ... per thread

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 4x4x1 MFMA whose B operand is lane group g (lanes 16 g .. 16 g + 15) of b, broadcast to
// all 16 blocks (BLGP = 4 + g; g must fold to a constant)
__device__ __forceinline__ f32x4 mfma4_bcast(float a, float b, f32x4 c, int g) {
  switch (g) {
    case 0: return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 4);
    case 1: return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 5);
    case 2: return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 6);
    default: return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 7);
  }
}

template <int NC>
__global__ __launch_bounds__(256, 2) void convt2_narrow_mfma(NarrowArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) float xs[NM_HR * NM_RS];
  __shared__ __attribute__((aligned(16))) float wl[NM_CH * 256];  // [c][r][lane] (pack_narrow order)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_c = (a.W + NM_TC - 1) / NM_TC, tiles_r = (a.H + NM_TR - 1) / NM_TR;
  const int per_img = tiles_c * tiles_r;
  const int co = lane & 3;
  // this lane's pixel in each group (tile coords): row 4 wid + lane / 16, col 16 g + lane % 16
  const int pr = 4 * wid + (lane >> 4), pc = lane & 15;
  // Persistent over (image, 16 x 32 tile) with the next channel chunk's halo and weights
  // loaded into registers while the current chunk's MFMAs run (the one-shot grid of 1024
  // blocks ran a 3-blocks-per-CU round plus a 1-block tail, every chunk's loads exposed).
  float4 stage[NM_XPT];
  float4 wv[4];
  // this thread's halo slots of the tile being prefetched: element offset of (pixel, channel
  // quad tid % 4) within the image, or -1 outside it -- computed once per tile, so a chunk's
  // prefetch is one add per load (the per-chunk index arithmetic was 1.6 VALU per MFMA, and
  // fp32 MFMA and VALU share the issue port)
  int xo[NM_XPT], sxo[NM_XPT];  // ... and its slots' LDS offsets (fixed per thread)
  const int q4 = 4 * (tid & 3);
#pragma unroll
  for (int t = 0; t < NM_XPT; ++t) {
    const int pix = (tid + 256 * t) >> 2, hr = pix / NM_HC;
    sxo[t] = hr * NM_RS + (pix - hr * NM_HC) * NM_LD + q4;
  }
  auto set_tile = [&](int r0, int c0p) {
#pragma unroll
    for (int t = 0; t < NM_XPT; ++t) {
      const int e = tid + 256 * t, pix = e >> 2;
      const int hr = pix / NM_HC, hc = pix - hr * NM_HC;
      const int ih = r0 - 1 + hr, iw = c0p - 1 + hc;
      xo[t] = (e < NM_XQ && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                  ? ih * (int)a.xsh + iw * (int)a.xsw + q4
                  : -1;
    }
  };
  auto load_chunk = [&](const float* xb, int ch0) {
    const bool cok = ch0 + q4 < a.C;
#pragma unroll
    for (int t = 0; t < NM_XPT; ++t) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && xo[t] >= 0) v = *reinterpret_cast<const float4*>(xb + xo[t] + ch0);
      stage[t] = v;
    }
    // weights: this chunk's [c][r][lane] slice of the pack, contiguous (c >= C -> 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * (tid + 256 * q);  // float index within the chunk's 16 x 256
      wv[q] = ch0 + (e >> 8) < a.C ? *reinterpret_cast<const float4*>(a.w + (size_t)ch0 * 256 + e)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto tile_of = [&](int t, int& b, int& r0, int& c0p) {
    b = t / per_img;
    const int trem = t - b * per_img, tr = trem / tiles_c;
    r0 = tr * NM_TR;
    c0p = (trem - tr * tiles_c) * NM_TC;
  };
  // work item = (tile, input-channel split): item = tile * splits + split.  Small grids
  // (G's 32 x 32 -> 64 x 64 image layer: 64 tiles) split the channel sum over blocks so the
  // chip is filled; the raw partial sums then go to a slab reduced in split order.
  const int items = ntiles * a.splits;
  auto item_of = [&](int it, int& t, int& cb, int& ce) {
    t = it / a.splits;
    cb = (it - t * a.splits) * a.cps;
    ce = min(a.C, cb + a.cps);
  };
  int it = blockIdx.x;
  if (it >= items) return;
  const float* xb_next;
  {
    int t, cb, ce, b, r0, c0p;
    item_of(it, t, cb, ce);
    tile_of(t, b, r0, c0p);
    set_tile(r0, c0p);
    xb_next = a.x + (long long)b * a.xsb;
    load_chunk(xb_next, cb);
  }
  for (; it < items; it += gridDim.x) {
    int t, cb, ce, b, r0, c0p;
    item_of(it, t, cb, ce);
    tile_of(t, b, r0, c0p);
    f32x4 acc[2][4];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[g][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch0 = cb; ch0 < ce; ch0 += NM_CH) {
      const int nch = min(NM_CH, ce - ch0);
      __syncthreads();  // previous chunk's (or tile's) LDS reads are done
#pragma unroll
      for (int q = 0; q < NM_XPT; ++q) {
        const int e = tid + 256 * q;
        if (e < NM_XQ) *reinterpret_cast<float4*>(xs + sxo[q]) = stage[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(wl + 4 * (tid + 256 * q)) = wv[q];
      __syncthreads();
      // the next chunk (or the next tile's first chunk) into registers during the MFMAs
      if (ch0 + NM_CH < ce) {
        load_chunk(xb_next, ch0 + NM_CH);
      } else if (it + (int)gridDim.x < items) {
        int t2, cb2, ce2, b2, r2, c2;
        item_of(it + (int)gridDim.x, t2, cb2, ce2);
        tile_of(t2, b2, r2, c2);
        set_tile(r2, c2);
        xb_next = a.x + (long long)b2 * a.xsb;
        load_chunk(xb_next, cb2);
      }
      for (int c4 = 0; c4 < nch / 4; ++c4) {
        float4 xv[2][3][3];
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v)
              xv[g][u][v] = *reinterpret_cast<const float4*>(xs + (pr + u) * NM_RS + (16 * g + pc + v) * NM_LD + 4 * c4);
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          // B operands: 4 registers of 4 taps each (one ds_read_b32 apiece: 64 distinct
          // words); the MFMA's BLGP = 4 + g broadcasts lane group g (tap 4 r + g, co = lane % 4)
          // to all 16 blocks
          float wr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) wr[r] = wl[((4 * c4 + cc) * 4 + r) * 64 + lane];
          // (th, tw) outermost: 8 consecutive MFMAs on 8 different accumulators
#pragma unroll
          for (int th = 0; th < 2; ++th)
#pragma unroll
            for (int tw = 0; tw < 2; ++tw)
#pragma unroll
              for (int ph = 0; ph < 2; ++ph)
#pragma unroll
                for (int pw = 0; pw < 2; ++pw) {
                  const int tap = (2 * th + 1 - ph) * 4 + (2 * tw + 1 - pw);
#pragma unroll
                  for (int g = 0; g < 2; ++g) {
                    const float4 xq = xv[g][ph - th + 1][pw - tw + 1];
                    const float xa = cc == 0 ? xq.x : cc == 1 ? xq.y : cc == 2 ? xq.z : xq.w;
                    acc[g][ph * 2 + pw] = mfma4_bcast(xa, wr[tap >> 2], acc[g][ph * 2 + pw], tap & 3);
                  }
                }
        }
      }
    }
    if (co < NC && a.splits > 1) {  // raw partial sums, [split][b][co][oh][ow]
      float* sb = a.slab + ((long long)((it % a.splits) * a.B + b) * NC + co) * a.Ho * a.Wo;
      const int blk = lane >> 2;
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 4 * blk + i;
          const int gi = r0 + 4 * wid + (q >> 4), gj = c0p + 16 * g + (q & 15);
          if (gi >= a.H || gj >= a.W) continue;
#pragma unroll
          for (int ph = 0; ph < 2; ++ph)
#pragma unroll
            for (int pw = 0; pw < 2; ++pw)
              sb[(long long)(2 * gi + ph) * a.Wo + 2 * gj + pw] = acc[g][ph * 2 + pw][i];
        }
    } else if (co < NC) {
      const float wsc = a.wscale ? a.wscale[0] : 1.f;
      const float bv = a.bias ? a.bias[co] : 0.f;
      float* yb = a.y + (long long)b * a.ysb + (long long)co * a.ysc;
      const int blk = lane >> 2;  // this lane holds pixels 4 blk + i of each group, channel co
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 4 * blk + i;  // pixel index within the group (lane order)
          const int gi = r0 + 4 * wid + (q >> 4), gj = c0p + 16 * g + (q & 15);
          if (gi >= a.H || gj >= a.W) continue;
#pragma unroll
          for (int ph = 0; ph < 2; ++ph)
#pragma unroll
            for (int pw = 0; pw < 2; ++pw)
              yb[(long long)(2 * gi + ph) * a.ysh + (long long)(2 * gj + pw) * a.ysw] =
                  act_fwd(acc[g][ph * 2 + pw][i] * wsc + bv, a.act, a.alpha);
        }
    }
  }
}

// y = act(sum over splits of convt2_narrow_mfma's partial sums * wscale + bias), splits
// added in order (deterministic); one thread per output element, slab reads coalesced
__global__ __launch_bounds__(256) void narrow_split_reduce(NarrowArgs a) {
  const long long per = (long long)a.Ho * a.Wo, n = (long long)a.B * a.Cout * per;
  const float wsc = a.wscale ? a.wscale[0] : 1.f;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    float v = a.slab[e];
    for (int sp = 1; sp < a.splits; ++sp) v += a.slab[(long long)sp * n + e];
    const long long bc = e / per, pix = e - bc * per;
    const int b = (int)(bc / a.Cout), co = (int)(bc - (long long)b * a.Cout);
    const int oh = (int)(pix / a.Wo), ow = (int)(pix - (long long)oh * a.Wo);
    a.y[(long long)b * a.ysb + (long long)co * a.ysc + (long long)oh * a.ysh + (long long)ow * a.ysw] =
        act_fwd(v * wsc + (a.bias ? a.bias[co] : 0.f), a.act, a.alpha);
  }
}

// packed narrow-ConvT weights in MFMA B-operand lane order, [C][4][64]: register r of input
// channel ci holds, in lane l, W[ci][co = l % 4][tap = 4 r + l / 16] (co >= NC: 0, the
// MFMA's fourth column) -- lane group l / 16 is one tap, selected by the MFMA's BLGP
// broadcast (convt2_narrow_mfma)
__global__ void pack_narrow(const float* __restrict__ W, float* __restrict__ out, int C, int NC, long long s_in,
                            long long s_out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= C * 256) return;
  const int l = e & 63, r = (e >> 6) & 3, ci = e >> 8, co = l & 3, t = 4 * r + (l >> 4);
  out[e] = co < NC ? W[ci * s_in + co * s_out + t] : 0.f;
}

// Tiled pack for the layouts whose columns are one weight index (n = out_idx) and whose
// rows are (tap, in_idx) with in_idx fastest -- every pack on the FAST paths: a block
// moves a 32 in x 8 out x (<= 16 taps) brick through LDS, reading W in its own contiguous
// order (taps, then the smaller-stride index: 512 or 128 contiguous floats) and writing
// whole 128-B lines (32-float k runs) of the [N][K] image.
constexpr int PK_I = 32, PK_O = 8, PK_LD = PK_O * 17 + 1;  // odd row stride: conflict-free reads
__device__ __forceinline__ void pack_tiled_body(const PackArgs& a, int bx, int by, float* t) {  // t: [in][out][tap]
  const int KK = a.KH * a.KW;
  const int Nin = (int)a.fpci.d, Nout = a.N;
  const int i0 = bx * PK_I, o0 = by * PK_O;
  const bool in_fast = a.s_in < a.s_out;
  for (int e = threadIdx.x; e < PK_I * PK_O * 16; e += 256) {
    const int tap = e & 15;
    const int i = in_fast ? (e >> 4) & (PK_I - 1) : e >> 7;
    const int o = in_fast ? e >> 9 : (e >> 4) & (PK_O - 1);
    float val = 0.f;
    if (tap < KK && i0 + i < Nin && o0 + o < Nout)
      val = a.W[(long long)(i0 + i) * a.s_in + (long long)(o0 + o) * a.s_out + tap];
    t[i * PK_LD + o * 17 + tap] = val;
  }
  __syncthreads();
  const int K = a.K;
  for (int e = threadIdx.x; e < PK_I * PK_O * 16; e += 256) {
    const int i = e & (PK_I - 1), o = (e >> 5) & (PK_O - 1), tap = e >> 8;
    if (tap >= KK || i0 + i >= Nin || o0 + o >= Nout) continue;
    const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
    int phase = 0, kt;
    if (a.convt2) {  // tap (kh, kw) of phase (ph, pw) = (2th+1-ph, 2tw+1-pw)
      phase = (1 - (kh & 1)) * 2 + (1 - (kw & 1));
      kt = (kh >> 1) * 2 + (kw >> 1);
    } else {
      kt = a.flip ? (a.KH - 1 - kh) * a.KW + (a.KW - 1 - kw) : tap;
    }
    a.out[((size_t)phase * Nout + o0 + o) * K + (size_t)kt * Nin + i0 + i] = t[i * PK_LD + o * 17 + tap];
  }
}

__global__ __launch_bounds__(256) void pack_tiled(PackArgs a) {
  __shared__ float t[PK_I * PK_LD];
  pack_tiled_body(a, blockIdx.x, blockIdx.y, t);
}

// 4x4 taps, Nin % 32 == 0, Nout % 8 == 0 (every C2 pack): the same brick moved with
// float4s -- 4 taps per load (taps are the weight's contiguous index), 4 in-indices per
// store (the packed row's contiguous index) -- 4 loads + 4 stores per thread, all issued
// before their first use.
constexpr int P4_LD = PK_O * 16 + 4;  // [in][out][16 taps], 16-B aligned rows
__device__ __forceinline__ void pack_tiled16_body(const PackArgs& a, int bx, int by, float* t) {
  const int Nin = (int)a.fpci.d, Nout = a.N, K = a.K;
  const int i0 = bx * PK_I, o0 = by * PK_O;
  const bool in_fast = a.s_in < a.s_out;
  float4 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = threadIdx.x + 256 * r;  // float4 index in the brick
    const int tq = e & 3;
    const int i = in_fast ? (e >> 2) & (PK_I - 1) : e >> 5;
    const int o = in_fast ? e >> 7 : (e >> 2) & (PK_O - 1);
    v[r] = *reinterpret_cast<const float4*>(a.W + (long long)(i0 + i) * a.s_in + (long long)(o0 + o) * a.s_out +
                                            4 * tq);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = threadIdx.x + 256 * r;
    const int tq = e & 3;
    const int i = in_fast ? (e >> 2) & (PK_I - 1) : e >> 5;
    const int o = in_fast ? e >> 7 : (e >> 2) & (PK_O - 1);
    *reinterpret_cast<float4*>(t + i * P4_LD + o * 16 + 4 * tq) = v[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = threadIdx.x + 256 * r;
    const int iq = e & 7, o = (e >> 3) & (PK_O - 1), tap = e >> 6;
    const int kh = tap >> 2, kw = tap & 3;
    int phase = 0, kt;
    if (a.convt2) {  // tap (kh, kw) of phase (ph, pw) = (2th+1-ph, 2tw+1-pw)
      phase = (1 - (kh & 1)) * 2 + (1 - (kw & 1));
      kt = (kh >> 1) * 2 + (kw >> 1);
    } else {
      kt = a.flip ? 15 - tap : tap;
    }
    const float* src = t + (4 * iq) * P4_LD + o * 16 + tap;
    *reinterpret_cast<float4*>(a.out + ((size_t)phase * Nout + o0 + o) * K + (size_t)kt * Nin + i0 + 4 * iq) =
        make_float4(src[0], src[P4_LD], src[2 * P4_LD], src[3 * P4_LD]);
  }
}

__global__ __launch_bounds__(256) void pack_tiled16(PackArgs a) {
  __shared__ __attribute__((aligned(16))) float t[PK_I * P4_LD];
  pack_tiled16_body(a, blockIdx.x, blockIdx.y, t);
}

// Every stale weight layout of a net after its optimizer step in one launch (the repacks
// of a small model are ~10 us launches of ~1 us of work each): entry j owns blocks
// [first[j], first[j+1]) of a 1-D grid, its own (bx, by) brick grid and kernel body.
constexpr int PACK_BATCH = 16;
struct PackBatch {
  PackArgs a[PACK_BATCH];
  int kind[PACK_BATCH];  // 0: pack_tiled16, 1: pack_tiled
  int gx[PACK_BATCH];
  int first[PACK_BATCH + 1];
  int n;
};

__global__ __launch_bounds__(256) void pack_multi(PackBatch b) {
  __shared__ __attribute__((aligned(16))) float t[PK_I * (P4_LD > PK_LD ? P4_LD : PK_LD)];
  int j = 0;
  while (j + 1 < b.n && (int)blockIdx.x >= b.first[j + 1]) ++j;
  const int local = (int)blockIdx.x - b.first[j], bx = local % b.gx[j], by = local / b.gx[j];
  if (b.kind[j] == 0) pack_tiled16_body(b.a[j], bx, by, t);
  else pack_tiled_body(b.a[j], bx, by, t);
}

// ---------------------------------------------------------------- Adam writing the GEMM layouts
// The optimizer step (GLI:659, 712) rewrites every weight; the conv GEMMs read packed copies
// ([phase][N][K], tiled16 / t2d / narrow layouts above).  Re-reading each weight after Adam
// to repack it cost 8 B per weight element and a launch per net (pack_multi: 2.9 GB, 0.57 ms
// per C3 iteration); here the Adam kernel writes the packed copies of the values it has in
// registers.  Weight viewed [A][B][KK] (contiguous); per cached layout:
//   APK_TILED   out[((phase Nout + o) K + kt Nin + i)], (i, o) = (a, b) or (b, a), the tap
//               -> (phase, kt) map of pack_tiled_body (flip / 4 sub-pixel phases);
//   APK_T2D     out[(tap Cout + co) K + ci]  (G's 1x1 -> 4x4 first layer, pack_t2d);
//   APK_NARROW  out[ci 256 + (t >> 2) 64 + (t & 3) 16 + x 4 + co], x = 0..3 (pack_narrow).
// A tensor whose layouts are all 4x4-tap tiled with A, B multiples of 32 runs as 32 x 32 x 16
// bricks: Adam on the brick (coalesced 2-KB rows), the new values into LDS, then each layout
// written as float4 runs of 4 consecutive in-indices (pack_tiled16's store pattern); other
// tensors run the flat 4096-element blocks of adam_kernel with per-element scatters.
enum { APK_TILED = 0, APK_T2D = 1, APK_NARROW = 2 };
struct AdamPackT {
  float* out;
  int kind, in_is_a, A, B, KK, KW, flip, convt2, Nin, Nout, K, NC;
};
struct AdamPackTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  long long n;
  int brick, bricks_b, pk0, npk;
};
// 1024 threads: a brick's 4096 float4 (or a flat block's 16384 elements) are one pass of 4
// float4 loads per thread and array, all in flight together (two 68-KB blocks per CU)
constexpr int AP_MAXT = 24, AP_MAXP = 24, AP_BRICK = 32 * 32 * 16, AP_FLAT = 16384, AP_TLD = 32 * 17 + 4,
              AP_THREADS = 1024;
struct AdamPackBatch {
  AdamPackTensor t[AP_MAXT];
  AdamPackT pk[AP_MAXP];
  int first[AP_MAXT + 1];
  int cnt;
};

__device__ __forceinline__ long long apk_tiled_dst(const AdamPackT& t, int a, int b, int tap) {
  const int i = t.in_is_a ? a : b, o = t.in_is_a ? b : a;
  const int kh = tap / t.KW, kw = tap - kh * t.KW;
  int phase = 0, kt;
  if (t.convt2) {
    phase = (1 - (kh & 1)) * 2 + (1 - (kw & 1));
    kt = (kh >> 1) * 2 + (kw >> 1);
  } else {
    kt = t.flip ? t.KK - 1 - tap : tap;
  }
  return ((long long)phase * t.Nout + o) * t.K + (long long)kt * t.Nin + i;
}

// brick path: destination of element (a, b, tap) of a TILED or T2D layout
__device__ __forceinline__ long long apk_brick_dst(const AdamPackT& t, int a, int b, int tap) {
  if (t.kind == APK_T2D) return ((long long)tap * t.B + b) * t.K + a;
  return apk_tiled_dst(t, a, b, tap);
}

// element e (flat index of the [A][B][KK] weight) with its new value into one layout
__device__ __forceinline__ void apk_scatter(const AdamPackT& t, long long e, float val) {
  const int tap = (int)(e % t.KK);
  const long long r = e / t.KK;
  const int a = (int)(r / t.B), b = (int)(r - (long long)a * t.B);
  if (t.kind == APK_TILED) {
    t.out[apk_tiled_dst(t, a, b, tap)] = val;
  } else if (t.kind == APK_T2D) {
    t.out[((long long)tap * t.B + b) * t.K + a] = val;
  } else {
    const long long o = (long long)a * 256 + (tap >> 2) * 64 + (tap & 3) * 16 + b;
#pragma unroll
    for (int x = 0; x < 4; ++x) t.out[o + 4 * x] = val;
  }
}

__device__ __forceinline__ void adam_pack_flat(const AdamPackBatch& b, const AdamPackTensor& X, const AdamConst& k,
                                               int local, int tid);

// The call's step-counter increment rides on its last launch: every block computes with
// step + 1 (read at entry), and the last block to arrive stores it -- after every block of
// every launch of the call has read the old value (no separate increment launch ahead of the
// step).  The arrival ticket is the group's own word next to its counter (step[1], 0 between
// calls), so optimizer steps of different groups / optimizers / streams never share one.

__global__ __launch_bounds__(AP_THREADS) void adam_pack_kernel(AdamPackBatch b, const double* __restrict__ hyper,
                                                               float* step, int bump) {
  __shared__ float T[32 * AP_TLD];  // brick [a][b][tap]: b stride 17, a stride 548 (4 consecutive a: distinct banks)
  int j = 0;
  while (j + 1 < b.cnt && (int)blockIdx.x >= b.first[j + 1]) ++j;
  const AdamPackTensor X = b.t[j];
  const float st1 = step[0] + 1.f;
  const AdamConst k = adam_const(hyper, &st1);
  const int local = (int)blockIdx.x - b.first[j], tid = threadIdx.x;
  if (X.brick) {
    const AdamPackT& t0 = b.pk[X.pk0];
    const int B = t0.B, a0 = 32 * (local / X.bricks_b), b0 = 32 * (local % X.bricks_b);
    {  // 32 rows of 32 b x 16 taps (2 KB contiguous each)
      float4 P[4], G[4], M[4], V[4];
      long long off[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int jj = tid + AP_THREADS * u, al = jj >> 7, f = jj & 127;
        off[u] = ((long long)(a0 + al) * B + b0) * 16 + 4 * f;
        P[u] = *reinterpret_cast<const float4*>(X.p + off[u]);
        G[u] = *reinterpret_cast<const float4*>(X.g + off[u]);
        M[u] = *reinterpret_cast<const float4*>(X.m + off[u]);
        V[u] = *reinterpret_cast<const float4*>(X.v + off[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        adam_elem(k, G[u].x, P[u].x, M[u].x, V[u].x);
        adam_elem(k, G[u].y, P[u].y, M[u].y, V[u].y);
        adam_elem(k, G[u].z, P[u].z, M[u].z, V[u].z);
        adam_elem(k, G[u].w, P[u].w, M[u].w, V[u].w);
        *reinterpret_cast<float4*>(X.m + off[u]) = M[u];
        *reinterpret_cast<float4*>(X.v + off[u]) = V[u];
        *reinterpret_cast<float4*>(X.p + off[u]) = P[u];
        const int jj = tid + AP_THREADS * u, al = jj >> 7, f = jj & 127, bl = f >> 2, tq = f & 3;
        float* d = T + al * AP_TLD + bl * 17 + 4 * tq;
        d[0] = P[u].x; d[1] = P[u].y; d[2] = P[u].z; d[3] = P[u].w;
      }
    }
    __syncthreads();
    for (int q = 0; q < X.npk; ++q) {
      const AdamPackT& t = b.pk[X.pk0 + q];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // 32 x 16 x 8 float4 of 4 consecutive in-indices
        const int jj = tid + AP_THREADS * u, iq = jj & 7, tap = (jj >> 3) & 15, ol = jj >> 7;
        float4 v4;
        long long dst;
        if (t.in_is_a) {  // in = a: T[4 iq + c][ol][tap]
          const float* s = T + (4 * iq) * AP_TLD + ol * 17 + tap;
          v4 = make_float4(s[0], s[AP_TLD], s[2 * AP_TLD], s[3 * AP_TLD]);
          dst = apk_brick_dst(t, a0 + 4 * iq, b0 + ol, tap);
        } else {          // in = b: T[ol][4 iq + c][tap]
          const float* s = T + ol * AP_TLD + (4 * iq) * 17 + tap;
          v4 = make_float4(s[0], s[17], s[34], s[51]);
          dst = apk_brick_dst(t, a0 + ol, b0 + 4 * iq, tap);
        }
        *reinterpret_cast<float4*>(t.out + dst) = v4;
      }
    }
  } else {
    adam_pack_flat(b, X, k, local, tid);
  }
  if (bump) {
    __syncthreads();  // every wave of this block has read step[0]
    unsigned int* ticket = reinterpret_cast<unsigned int*>(step + 1);
    if (threadIdx.x == 0 && atomicAdd(ticket, 1u) == gridDim.x - 1) {
      step[0] = st1;
      atomicExch(ticket, 0u);
    }
  }
}

__device__ __forceinline__ void adam_pack_flat(const AdamPackBatch& b, const AdamPackTensor& X, const AdamConst& k,
                                               int local, int tid) {
  const long long e0 = (long long)local * AP_FLAT, e1 = min(X.n, e0 + AP_FLAT);
  const bool vec = (X.n & 3) == 0 && ((((uintptr_t)X.p | (uintptr_t)X.g | (uintptr_t)X.m | (uintptr_t)X.v) & 15) == 0);
  if (vec) {
    constexpr int U = AP_FLAT / (4 * AP_THREADS);
    float4 P[U], G[U], M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = e0 + 4 * (tid + AP_THREADS * u);
      if (i < e1) {
        P[u] = *reinterpret_cast<const float4*>(X.p + i);
        G[u] = *reinterpret_cast<const float4*>(X.g + i);
        M[u] = *reinterpret_cast<const float4*>(X.m + i);
        V[u] = *reinterpret_cast<const float4*>(X.v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = e0 + 4 * (tid + AP_THREADS * u);
      if (i < e1) {
        adam_elem(k, G[u].x, P[u].x, M[u].x, V[u].x);
        adam_elem(k, G[u].y, P[u].y, M[u].y, V[u].y);
        adam_elem(k, G[u].z, P[u].z, M[u].z, V[u].z);
        adam_elem(k, G[u].w, P[u].w, M[u].w, V[u].w);
        *reinterpret_cast<float4*>(X.m + i) = M[u];
        *reinterpret_cast<float4*>(X.v + i) = V[u];
        *reinterpret_cast<float4*>(X.p + i) = P[u];
        for (int q = 0; q < X.npk; ++q) {
          const AdamPackT& t = b.pk[X.pk0 + q];
          apk_scatter(t, i, P[u].x);
          apk_scatter(t, i + 1, P[u].y);
          apk_scatter(t, i + 2, P[u].z);
          apk_scatter(t, i + 3, P[u].w);
        }
      }
    }
  } else {
    for (long long i = e0 + tid; i < e1; i += AP_THREADS) {
      float p = X.p[i], m = X.m[i], v = X.v[i];
      adam_elem(k, X.g[i], p, m, v);
      X.m[i] = m;
      X.v[i] = v;
      X.p[i] = p;
      for (int q = 0; q < X.npk; ++q) apk_scatter(b.pk[X.pk0 + q], i, p);
    }
  }
}

// ---------------------------------------------------------------- host planning
enum { CFG_L = 0, CFG_M = 1, CFG_N = 2, CFG_S = 3 };

struct Plan {
  int mode = MODE_CONV;
  GemmArgs g{};
  int phases = 1;
  int cfg = CFG_L;
  bool av = false, bv = false, fast = false;
  // packing
  bool pack = false;
  const float* prepacked = nullptr;  // caller-owned packed weights (skip packing)
  PackArgs pk{};
  size_t pack_floats = 0, slab_floats = 0;
  // WGRAD tap-major staging (taps_transpose): C of the GEMM -> workspace, then torch layout
  bool tap_stage = false;
  size_t tap_floats = 0;
  // narrow kernels (MODE_NARROW_T / MODE_NARROW_IN)
  NarrowArgs na{};
  long long pn_s_in = 0, pn_s_out = 0;  // narrow pack strides
  // one-output dense layer (MODE_DENSE1): which = 0 fwd, 1 dgrad, 2 wgrad
  DenseArgs da{};
  int dense_op = 0;
  bool img_in = false;  // MODE_NARROW_IN on the windowed kernel (conv_img_in)
  // BatchNorm moments in the vector epilogue (rgan_conv_fwd_bn): caller's [S][2][C] buffer,
  // equal batch segments whose statistics are kept apart, and whether the launch wrote them
  double* bn_part = nullptr;
  int bn_segs = 1;
  bool bn_fused = false;
  // producer post-op (rgan_conv_post): requested, and whether this plan applies it
  const RganPost* post = nullptr;
  bool post_fused = false;
};

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static void tile_dims(int cfg, int& bm, int& bn) {
  bm = cfg == CFG_N ? 256 : (cfg == CFG_S ? 64 : 128);
  bn = cfg == CFG_L ? 128 : (cfg == CFG_M || cfg == CFG_S ? 64 : 32);
}

// fewest k steps (of BK) per split (round-4 A/B against 2 / 8 / 16: profiles/round4_split_planner_ab.txt)
constexpr int SPLIT_MINK = 4;

// opt-in fp32-on-bf16x6 GEMMs (rgan_set_gemm_emulation)
static std::atomic<int> g_emu{0};
static bool emu_bf16x6() { return g_emu.load(std::memory_order_relaxed) == 1; }

// below SMALL_GEMM_FLOPS, smaller tiles instead of a >= SMALL_SPLITS-way split of 128 x 128
// ones: 64 x 64 for the forward / data gradients (round 5: four times the tiles, a quarter of
// the splits, half the slab bytes per output; C4 3.74 -> 3.53 ms/step, run r5q) and for the
// weight gradients of <= 64 output channels (whose 128-row tiles were half empty: C4 9339 /
// 9357 -> 9427 / 9443 img/s, run r5aa), 128 x 64 for the other weight gradients (C4 3.93 ->
// 3.85 ms/step, run r4v; on 64 x 64 they measured slower, run r5r)
constexpr double SMALL_GEMM_FLOPS = 4e9;
constexpr int SMALL_SPLITS = 4;

static void choose_tiling(Plan& p) {
  GemmArgs& g = p.g;
  p.cfg = g.N <= 32 ? CFG_N : (g.N <= 64 ? CFG_M : CFG_L);
  // small forward / data-gradient GEMMs with N <= 64: 64 x 64 tiles, twice the tiles of
  // 128 x 64 and half its splits (C4 3.535 -> 3.43 ms/step, run r5r; weight gradients stay
  // on 128 x 64: 3.535 -> 3.55 with them moved too)
  if (p.cfg == CFG_M && p.mode != MODE_WGRAD && 2.0 * g.M * g.N * g.K * p.phases < SMALL_GEMM_FLOPS && !emu_bf16x6())
    p.cfg = CFG_S;
  // the weight gradient of a thin input layer (N = taps x <= 3 channels <= 32, M = Cout <= 64:
  // arch 1's Conv3x3 3 -> 64, GLI:260): a 256-row tile would be >= 75 % empty rows (round 6)
  if (p.cfg == CFG_N && p.mode == MODE_WGRAD && g.M <= 64 && !emu_bf16x6()) p.cfg = CFG_S;
  // a thin-M forward with many outputs (arch 1's G input Linear, z -> 4 x 4 x 512 as a 1 x 1 conv
  // over a 1 x 1 map, M = B = 32): 64 x 64 tiles, 128 blocks instead of 64 half-empty 128 x 128
  // ones -- 6.2 us per C4 call vs 15.8 (and vs 13.5 for a VALU kernel with LDS-staged rows;
  // round 6, tools/dense_micro.py)
  if (p.mode == MODE_CONV && g.M <= 64 && g.N >= 4096 && g.K <= 512 && !emu_bf16x6()) p.cfg = CFG_S;
  // ... and its weight gradient (M = 8192 outputs, K = B = 32 pixel rows): 64 x 64 tiles, 256 blocks of
  // one k tile instead of 64 -- 6.4 us per C4 call with the bias vs 19.5 (and vs 12.1 for a VALU
  // kernel with LDS-staged rows, round 6)
  if (p.mode == MODE_WGRAD && g.K <= 64 && g.M >= 4096 && !emu_bf16x6()) p.cfg = CFG_S;
  if (p.cfg == CFG_L) {
    const long long t = (long long)ceil_div(g.M, 128) * ceil_div(g.N, 128) * p.phases;
    const int nk = ceil_div(g.K, BK);
    // small GEMMs (arch 1 at 32x32: 0.1-1.5 GFLOP) that would split K 4+ ways: more tiles,
    // fewer splits and less reduce (128 x 64: C4 4.03 -> 3.92 ms/step, run r4t; 64 x 64 for
    // CONV / CONVT2: 3.74 -> 3.53, run r5q); at C1's 8.6-GFLOP GEMMs the same swap loses
    // (round-4 run r4c)
    const double flops = 2.0 * g.M * g.N * g.K * p.phases;
    // (not under the bf16x6 emulation, whose kernels are 128 x 128)
    if (flops < SMALL_GEMM_FLOPS && t * SMALL_SPLITS <= SPLIT_TARGET && nk >= 4 * SMALL_SPLITS && !emu_bf16x6())
      p.cfg = p.mode == MODE_WGRAD && g.M > 64 ? CFG_M : CFG_S;
  }
  int bm, bn;
  tile_dims(p.cfg, bm, bn);
  const int tiles_m = ceil_div(g.M, bm), tiles_n = ceil_div(g.N, bn);
  g.tiles_n = tiles_n;
  const long long tiles = (long long)tiles_m * tiles_n * p.phases;
  const int nk = ceil_div(g.K, BK);
  int splits = 1;
  // two resident 256-thread blocks per CU on 256 CUs (round-1 sweep of this target: 256 / 384 / 768 /
  // 1024 all lost to 512, profiles/round1_splitk_target_sweep.txt)
  constexpr long long target = SPLIT_TARGET;
  if (tiles < target) {
    splits = (int)((target + tiles - 1) / tiles);
    splits = std::min(splits, std::max(1, nk / SPLIT_MINK));
    splits = std::min(splits, 256);
    // bound the slab to 256 MiB
    while (splits > 1 && (size_t)splits * g.M * g.N * p.phases > (size_t)64 << 20) --splits;
  }
  const int per = ceil_div(nk, splits);
  g.ksplit = per * BK;
  g.splits = ceil_div(g.K, g.ksplit);
  if (g.splits < 1) g.splits = 1;
  // [phase][split][M][N] (splitk_reduce), sized in whole tiles
  p.slab_floats = g.splits > 1 ? (size_t)g.splits * tiles * bm * bn : 0;
}

static OutMap make_out(int gh, int gw, int step, long long sb, long long sh, long long sw, int nkh,
                       int nkw, int nc, long long th, long long tw, long long tc) {
  OutMap o;
  o.fgw = FastDiv(gw);
  o.fghw = FastDiv((uint32_t)gh * gw);
  o.step = step;
  o.sb = sb; o.sh = sh; o.sw = sw;
  o.fnc = FastDiv(nc);
  o.fnkw = FastDiv(nkw);
  (void)nkh;
  o.th = th; o.tw = tw; o.tc = tc;
  return o;
}

static Img make_img(const float* p, int H, int W, int C, const long long* s /* b,c,h,w */) {
  Img im;
  im.p = p; im.H = H; im.W = W; im.C = C;
  im.sb = s[0]; im.sc = s[1]; im.sh = s[2]; im.sw = s[3];
  // size-1 spatial dims: only index 0 is ever read, so give them the dense NHWC stride (z as
  // [B][C][1][1] -- G's first layer -- then qualifies for the vector/FAST loaders)
  if (W == 1 && im.sc == 1) im.sw = C;
  if (H == 1 && im.sc == 1) im.sh = (long long)W * im.sw;
  return im;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static bool vec_img_ok(const Img& im) {
  return im.sc == 1 && im.C % 4 == 0 && im.sh % 4 == 0 && im.sw % 4 == 0 && im.sb % 4 == 0 &&
         aligned16(im.p);
}

// bytes spanned by an image of `batch` samples (largest element offset + 1)
static long long img_span_bytes(const Img& im, int batch) {
  return 4LL * ((long long)(batch - 1) * im.sb + (long long)(im.H - 1) * im.sh + (long long)(im.W - 1) * im.sw +
                (long long)(im.C - 1) * im.sc + 1);
}

// FAST-path eligibility (see gemm_kernel): call after choose_tiling
static void set_fast(Plan& p, int batch) {
  GemmArgs& g = p.g;
  p.fast = false;
  g.im_buf = 0;
  if (p.mode == MODE_WGRAD && !p.bv) {  // the scalar im2col gathers through a descriptor (element offsets < 2^29)
    const long long im_bytes = img_span_bytes(g.im, batch);
    if (im_bytes <= FAST_MAX_BYTES / 4 && g.im.sb >= 0 && g.im.sh >= 0 && g.im.sw >= 0 && g.im.sc >= 0) {
      g.im_bytes = (int)im_bytes;
      g.im_buf = 1;
    }
  }
  if (!p.av || !p.bv || g.K % BK != 0) return;
  int bm, bn;
  tile_dims(p.cfg, bm, bn);
  const long long a_bytes = img_span_bytes(g.a, batch);
  if (a_bytes > FAST_MAX_BYTES) return;
  if (p.mode != MODE_WGRAD) {
    const long long bw = 4LL * g.K * g.N * p.phases;
    if ((int)g.fC.d % BK != 0 || bw > FAST_MAX_BYTES) return;
    g.a_bytes = (int)a_bytes;
    g.bw_bytes = (int)(4LL * g.K * g.N);
  } else {
    const long long im_bytes = img_span_bytes(g.im, batch);
    if (im_bytes > FAST_MAX_BYTES) return;
    if (g.a.sh != (long long)g.a.W * g.a.sw || g.a.sb != (long long)g.a.H * g.a.sh) return;
    // a B tile is one tap's BN channels, or BN / Cin <= 4 whole taps of one kernel row
    const int cin = g.im.C;
    if (cin % bn != 0 && !(bn % cin == 0 && cin % 4 == 0 && bn / cin <= 4 && g.KW % (bn / cin) == 0))
      return;
    g.a_bytes = (int)a_bytes;
    g.im_bytes = (int)im_bytes;
  }
  p.fast = true;
}

static void set_pack(Plan& p, const float* W, const float* scale, int K, int N, int pci, int pkw,
                     int nco, int nkw, long long s_in, long long s_out, long long s_kh, long long s_kw,
                     int KH, int KW, int flip, int convt2) {
  p.pack = true;
  p.g.wscale = scale;
  PackArgs& a = p.pk;
  a.W = W; a.K = K; a.N = N; a.phases = p.phases;
  a.fpci = FastDiv(pci); a.fpkw = FastDiv(pkw);
  a.fnco = FastDiv(nco); a.fnkw = FastDiv(nkw);
  a.s_in = s_in; a.s_out = s_out; a.s_kh = s_kh; a.s_kw = s_kw;
  a.KH = KH; a.KW = KW; a.flip = flip; a.convt2 = convt2;
  p.pack_floats = (size_t)K * N * p.phases;
}

static bool desc_ok(const RganConv* d) {
  if (!d) return false;
  if (d->batch <= 0 || d->cin <= 0 || d->cout <= 0 || d->kh <= 0 || d->kw <= 0 || d->stride <= 0 ||
      d->pad < 0 || d->hin <= 0 || d->win <= 0 || d->hout <= 0 || d->wout <= 0 ||
      (d->transposed != 0 && d->transposed != 1))
    return false;
  // sizes bounded before any arithmetic on them (every product below stays in 64 bits)
  constexpr int DMAX = 1 << 24, KMAX = 256;
  if (d->batch > DMAX || d->cin > DMAX || d->cout > DMAX || d->hin > DMAX || d->win > DMAX || d->hout > DMAX ||
      d->wout > DMAX || d->kh > KMAX || d->kw > KMAX || d->stride > KMAX || d->pad > KMAX)
    return false;
  const long long hin = d->hin, win = d->win, kh = d->kh, kw = d->kw, st = d->stride, pad = d->pad;
  if (!d->transposed) {
    if (hin + 2 * pad < kh || win + 2 * pad < kw) return false;
    if (d->hout != (hin + 2 * pad - kh) / st + 1) return false;
    if (d->wout != (win + 2 * pad - kw) / st + 1) return false;
  } else {
    if (d->hout != (hin - 1) * st - 2 * pad + kh) return false;
    if (d->wout != (win - 1) * st - 2 * pad + kw) return false;
  }
  // 32-bit index space for the GEMM dims
  if ((long long)d->batch * d->hout * d->wout >= (1LL << 31)) return false;
  if ((long long)d->batch * d->hin * d->win >= (1LL << 31)) return false;
  // kernel / channel sizes whose products (K = taps x channels, N = taps x outputs of the 1x1
  // expansion, packed-weight sizes) stay in int; non-negative strides whose extents stay far
  // inside 64-bit offsets (the host-side fuzz of tests/test_host_asan.py)
  const long long taps = kh * kw;
  if (taps * d->cin >= (1LL << 31) || taps * d->cout >= (1LL << 31) || (long long)d->cin * d->cout * taps >= (1LL << 40))
    return false;
  constexpr long long SMAX = 1LL << 40;
  double xext = 0.0, yext = 0.0;
  const int xd[4] = {d->batch, d->cin, d->hin, d->win}, yd[4] = {d->batch, d->cout, d->hout, d->wout};
  for (int i = 0; i < 4; ++i) {
    if (d->xs[i] < 0 || d->xs[i] > SMAX || d->ys[i] < 0 || d->ys[i] > SMAX) return false;
    xext += (double)(xd[i] - 1) * (double)d->xs[i];
    yext += (double)(yd[i] - 1) * (double)d->ys[i];
  }
  return xext < (double)SMAX && yext < (double)SMAX;
}

static bool is_k4s2p1(const RganConv* d) {
  return d->kh == 4 && d->kw == 4 && d->stride == 2 && d->pad == 1;
}

static bool vec_nhwc(const float* p, const long long* s, int C) {
  return s[1] == 1 && C % 4 == 0 && s[0] % 4 == 0 && s[2] % 4 == 0 && s[3] % 4 == 0 && aligned16(p);
}

// k4 s2 p1 ConvTranspose2d over input grid x (channels C, NHWC) with nc <= 4 outputs;
// weight element (in ci, out co, kh, kw) at w[ci * s_in + co * s_out + kh * 4 + kw]
static bool plan_narrow_t(Plan& p, int batch, const float* x, const long long* xs, int H, int W, int C,
                          const float* w, long long s_in, long long s_out, int nc, float* y, const long long* ys,
                          const float* wscale, const float* bias, int act, float alpha) {
  if (nc > 4 || !vec_nhwc(x, xs, C)) return false;
  p.mode = MODE_NARROW_T;
  NarrowArgs& a = p.na;
  a.x = x; a.xsb = xs[0]; a.xsc = xs[1]; a.xsh = xs[2]; a.xsw = xs[3];
  a.B = batch; a.H = H; a.W = W; a.C = C;
  a.w = w; a.y = y; a.ysb = ys[0]; a.ysc = ys[1]; a.ysh = ys[2]; a.ysw = ys[3];
  a.Ho = 2 * H; a.Wo = 2 * W; a.Cout = nc; a.stride = 2; a.pad = 1;
  a.bias = bias; a.wscale = wscale; a.act = act; a.alpha = alpha;
  p.pack = true;
  p.pack_floats = (size_t)C * 256;
  p.pn_s_in = s_in; p.pn_s_out = s_out;
  // channel splits when the tiles alone cannot fill the chip (two resident blocks per CU)
  const long long ntiles = (long long)batch * ceil_div(H, NM_TR) * ceil_div(W, NM_TC);
  const int chunks = ceil_div(C, NM_CH);
  int splits = 1;
  if (ntiles < 256)
    splits = (int)std::min<long long>(std::min(chunks, NARROW_MAX_SPLITS),
                                      ceil_div(512, (int)std::max<long long>(ntiles, 1)));
  a.cps = ceil_div(chunks, std::max(splits, 1)) * NM_CH;
  a.splits = ceil_div(C, a.cps);
  a.slab = nullptr;
  p.slab_floats = a.splits > 1 ? (size_t)a.splits * batch * nc * 4 * H * W : 0;
  p.pk.W = w;
  return true;
}

// Conv2d with a 4x4 kernel and <= 4 input channels (any input strides)
static bool plan_narrow_in(Plan& p, const RganConv* d, const float* x, const float* w, const float* wscale,
                           const float* bias, float* y, int act, float alpha) {
  if (d->transposed || d->cin > 4 || d->kh != 4 || d->kw != 4) return false;
  p.mode = MODE_NARROW_IN;
  // the wave-tiled kernel (conv_img_in): k4 s2 p1 halving of an image with <= 3 channels,
  // 128-channel tiles, NHWC output, 32-pixel wave tiles (row segments or two 16-wide rows),
  // 16-B window pieces (input rows contiguous and 16-B aligned)
  const long long xext = 4 * (1 + (d->batch - 1) * d->xs[0] + (d->cin - 1) * d->xs[1] + (d->hin - 1) * d->xs[2] +
                              (d->win - 1) * d->xs[3]);
  const long long yext = 4 * (1 + (d->batch - 1) * d->ys[0] + (d->cout - 1) * d->ys[1] + (d->hout - 1) * d->ys[2] +
                              (d->wout - 1) * d->ys[3]);
  p.img_in = d->stride == 2 && d->pad == 1 && d->hout * 2 == d->hin &&
             d->wout * 2 == d->win && d->cin <= 3 && (d->cout % 128 == 0 || (d->cin == 3 && d->cout % 32 == 0)) &&
             vec_nhwc(y, d->ys, d->cout) &&
             (d->wout == 16 || d->wout % 32 == 0) && ((long long)d->batch * d->hout * d->wout / 32) < (1LL << 31) &&
             d->xs[3] == 1 && d->xs[0] % 4 == 0 && d->xs[1] % 4 == 0 && d->xs[2] % 4 == 0 && d->xs[0] >= 0 &&
             d->xs[1] >= 0 && d->xs[2] >= 0 && ((uintptr_t)x & 15) == 0 && xext < (1LL << 31) && yext < (1LL << 31);
  NarrowArgs& a = p.na;
  a.x = x; a.xsb = d->xs[0]; a.xsc = d->xs[1]; a.xsh = d->xs[2]; a.xsw = d->xs[3];
  a.B = d->batch; a.H = d->hin; a.W = d->win; a.C = d->cin;
  a.w = w; a.y = y; a.ysb = d->ys[0]; a.ysc = d->ys[1]; a.ysh = d->ys[2]; a.ysw = d->ys[3];
  a.Ho = d->hout; a.Wo = d->wout; a.Cout = d->cout; a.stride = d->stride; a.pad = d->pad;
  a.bias = bias; a.wscale = wscale; a.act = act; a.alpha = alpha;
  a.x_bytes = (int)std::min(xext, (1LL << 31) - 1);
  a.y_bytes = (int)std::min(yext, (1LL << 31) - 1);
  p.pack = false;
  return true;
}

// Conv2d 3x3 stride 1 with nc <= 4 outputs over an NHWC input of C channels (C % 16 == 0):
// conv3_narrow_out.  Weight element (out n, in c, tap t) at w[n w_sn + c w_sc + (flip ? 8 - t : t)].
static bool plan_narrow3_out(Plan& p, int batch, const float* x, const long long* xs, int H, int W, int C,
                             const float* w, long long w_sn, long long w_sc, int flip, int nc, float* y,
                             const long long* ys, int Ho, int Wo, int pad, const float* wscale, const float* bias,
                             int act, float alpha) {
  if (nc > 4 || C < 4 || C > N3_MAXC || (C & (C - 1)) || xs[1] != 1 || xs[0] % 4 || xs[2] % 4 || xs[3] % 4 ||
      !aligned16(x))
    return false;
  if (Ho != H + 2 * pad - 2 || Wo != W + 2 * pad - 2) return false;
  p.mode = MODE_NARROW3;
  NarrowArgs& a = p.na;
  a.x = x; a.xsb = xs[0]; a.xsc = xs[1]; a.xsh = xs[2]; a.xsw = xs[3];
  a.B = batch; a.H = H; a.W = W; a.C = C;
  a.w = w; a.w_sn = w_sn; a.w_sc = w_sc; a.w_flip = flip;
  a.y = y; a.ysb = ys[0]; a.ysc = ys[1]; a.ysh = ys[2]; a.ysw = ys[3];
  a.Ho = Ho; a.Wo = Wo; a.Cout = nc; a.stride = 1; a.pad = pad;
  a.bias = bias; a.wscale = wscale; a.act = act; a.alpha = alpha;
  // pixels per wave: 64 / (C / 4) per step; enough steps to spread the per-wave weight loads,
  // few enough to leave >= ~8 waves per CU
  const long long P = (long long)batch * Ho * Wo, pw = 64 / (C / 4);
  a.rows = (int)std::max(1LL, std::min(16LL, P / (pw * 2048)));
  // 32-bit pixel indices and a buffer descriptor over x's extent
  const long long ext = ((long long)(batch - 1) * xs[0] + (long long)(H - 1) * xs[2] + (long long)(W - 1) * xs[3] + C) * 4;
  if (P + 64LL * (a.rows + 2) >= (1LL << 31) || ext >= 0x7ffffff0LL || xs[0] < 0 || xs[2] < 0 || xs[3] < 0) return false;
  a.x_bytes = (int)ext;
  p.pack = false;
  return true;
}

// weight gradient of a 3x3 stride-1 pad-1 Conv2d with <= 4 output channels (wgrad3_narrow + the
// WGRAD split reduce)
static bool plan_wgrad3_narrow(Plan& p, const RganConv* d, const float* x, const float* dy, float* dw) {
  if (d->transposed || d->kh != 3 || d->kw != 3 || d->stride != 1 || d->pad != 1 || d->cout > 4)
    return false;
  const int cw = d->cin;
  if (cw % 4 || 9 * (cw / 4) > 1024) return false;
  // R whole output rows per block, staged in LDS
  const int R = std::max(1, std::min(d->hout, N3W_PIX / std::max(1, d->wout)));
  if (wgrad3_lds_bytes(R, d->wout, cw, d->cout) > 64 * 1024) return false;
  p.mode = MODE_NARROW3W;
  NarrowArgs& a = p.na;
  a.x = x; a.xsb = d->xs[0]; a.xsc = d->xs[1]; a.xsh = d->xs[2]; a.xsw = d->xs[3];
  a.dy = dy; a.dsb = d->ys[0]; a.dsc = d->ys[1]; a.dsh = d->ys[2]; a.dsw = d->ys[3];
  a.B = d->batch; a.H = d->hin; a.W = d->win; a.C = d->cin;
  a.Ho = d->hout; a.Wo = d->wout; a.Cout = d->cout; a.stride = 1; a.pad = d->pad;
  const long long P = (long long)d->batch * d->hout * d->wout;
  a.rows = R;
  a.chunks = d->batch * ceil_div(d->hout, R);
  p.slab_floats = (size_t)a.chunks * d->cout * 9 * d->cin;
  // the reduce: the WGRAD GEMM's [split][M = cout][N = (kh, kw, ci)] slab into torch layout
  GemmArgs& g = p.g;
  g.M = d->cout; g.N = 9 * d->cin; g.K = (int)P; g.splits = a.chunks;
  g.C = dw; g.bias = nullptr; g.wscale = nullptr; g.act = RGAN_ACT_NONE; g.alpha = 0.f; g.pmode = 0;
  g.out = make_out(1, 1, 1, (long long)d->cin * 9, 0, 0, 3, 3, d->cin, 3, 1, 9);
  p.phases = 1;
  p.pack = false;
  return true;
}

// Conv2d(C, 1, k, 1, 0) over exactly a k x k map (x strides d->xs; y / dy at b * ys[0])
static bool plan_dense1(Plan& p, const RganConv* d, int op, const float* x, const float* w, const float* wscale,
                        const float* bias, float* y, float* out, int act, float alpha) {
  if (d->transposed || d->cout != 1 || d->hout != 1 || d->wout != 1 || d->pad != 0 || d->kh != d->hin ||
      d->kw != d->win)
    return false;
  if ((long long)d->batch * d->cin * d->hin * d->win >= (1LL << 31)) return false;
  p.mode = MODE_DENSE1;
  p.dense_op = op;
  p.pack = false;
  if (op != 2) {
    // filter packed in e order: Wp[(kh,kw,ci)] = W[0][ci][kh][kw] (the conv forward pack)
    const int KK = d->kh * d->kw;
    set_pack(p, w, wscale, KK * d->cin, 1, d->cin, d->kw, 1, 1, KK, (long long)d->cin * KK, d->kw, 1, d->kh,
             d->kw, 0, 0);
  }
  DenseArgs& a = p.da;
  a.x = x; a.xsb = d->xs[0]; a.xsc = d->xs[1]; a.xsh = d->xs[2]; a.xsw = d->xs[3];
  a.w = w; a.wscale = wscale; a.bias = bias; a.y = y; a.ysb = d->ys[0]; a.out = out;
  a.B = d->batch; a.C = d->cin; a.HW = d->hin * d->win; a.E = a.C * a.HW;
  a.fc = FastDiv(d->cin); a.fw = FastDiv(d->win);
  a.act = act; a.alpha = alpha;
  return true;
}

// forward GEMM over the conv's input x producing y (conv or transposed conv)
static int plan_fwd(const RganConv* d, const float* x, const float* w, const float* wscale,
                    const float* bias, float* y, int act, float alpha, Plan& p) {
  if (!desc_ok(d)) return RGAN_EINVAL;
  GemmArgs& g = p.g;
  const int KK = d->kh * d->kw;
  if (d->transposed && is_k4s2p1(d) && d->hout == 2 * d->hin && d->wout == 2 * d->win &&
      plan_narrow_t(p, d->batch, x, d->xs, d->hin, d->win, d->cin, w, (long long)d->cout * 16, 16, d->cout, y, d->ys,
                    wscale, bias, act, alpha))
    return 0;
  if (plan_narrow_in(p, d, x, w, wscale, bias, y, act, alpha)) return 0;
  if (plan_dense1(p, d, 0, x, w, wscale, bias, y, nullptr, act, alpha)) return 0;
  if (!d->transposed && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->cout <= 4 &&
      plan_narrow3_out(p, d->batch, x, d->xs, d->hin, d->win, d->cin, w, (long long)d->cin * 9, 9, 0, d->cout, y,
                       d->ys, d->hout, d->wout, d->pad, wscale, bias, act, alpha))
    return 0;
  g.a = make_img(x, d->hin, d->win, d->cin, d->xs);
  g.C = y; g.bias = bias; g.act = act; g.alpha = alpha;
  if (!d->transposed) {
    p.mode = MODE_CONV;
    g.M = d->batch * d->hout * d->wout; g.N = d->cout; g.K = KK * d->cin;
    g.KH = d->kh; g.KW = d->kw; g.stride = d->stride; g.pad = d->pad;
    g.fgw = FastDiv(d->wout); g.fghw = FastDiv((uint32_t)d->hout * d->wout);
    g.fC = FastDiv(d->cin); g.fKW = FastDiv(d->kw);
    g.out = make_out(d->hout, d->wout, 1, d->ys[0], d->ys[2], d->ys[3], 1, 1, d->cout, 0, 0, d->ys[1]);
    // Wp[(kh,kw,ci)][co] = W[co][ci][kh][kw]
    set_pack(p, w, wscale, g.K, g.N, d->cin, d->kw, d->cout, 1, KK, (long long)d->cin * KK, d->kw, 1,
             d->kh, d->kw, 0, 0);
  } else if (is_k4s2p1(d) && d->hout == 2 * d->hin && d->wout == 2 * d->win) {
    p.mode = MODE_CONVT2;
    p.phases = 4;
    g.M = d->batch * d->hin * d->win; g.N = d->cout; g.K = 4 * d->cin;
    g.KH = 4; g.KW = 4; g.stride = 2; g.pad = 1;
    g.fgw = FastDiv(d->win); g.fghw = FastDiv((uint32_t)d->hin * d->win);
    g.fC = FastDiv(d->cin); g.fKW = FastDiv(2);
    g.out = make_out(d->hin, d->win, 2, d->ys[0], d->ys[2], d->ys[3], 1, 1, d->cout, 0, 0, d->ys[1]);
    // ConvT weight [ci][co][kh][kw]
    set_pack(p, w, wscale, g.K, g.N, d->cin, 2, d->cout, 1, (long long)d->cout * 16, 16, 4, 1, 4, 4, 0, 1);
  } else if (d->hin == 1 && d->win == 1 && d->stride == 1 && d->pad == 0) {
    // 1x1 -> kh x kw expansion (G's first layer, GLI:336): plain GEMM, N = (oh, ow, co)
    p.mode = MODE_CONV;
    g.M = d->batch; g.N = KK * d->cout; g.K = d->cin;
    g.KH = 1; g.KW = 1; g.stride = 1; g.pad = 0;
    g.fgw = FastDiv(1); g.fghw = FastDiv(1);
    g.fC = FastDiv(d->cin); g.fKW = FastDiv(1);
    g.out = make_out(1, 1, 1, d->ys[0], 0, 0, d->kh, d->kw, d->cout, d->ys[2], d->ys[3], d->ys[1]);
    // Wp[ci][(oh,ow,co)] = W[ci][co][oh][ow]
    set_pack(p, w, wscale, g.K, g.N, d->cin, 1, d->cout, d->kw, (long long)d->cout * KK, KK, d->kw, 1,
             d->kh, d->kw, 0, 0);
  } else if (d->stride == 1) {
    // stride-1 transposed conv == conv with the flipped kernel and pad k-1-p
    p.mode = MODE_CONV;
    g.M = d->batch * d->hout * d->wout; g.N = d->cout; g.K = KK * d->cin;
    g.KH = d->kh; g.KW = d->kw; g.stride = 1; g.pad = d->kh - 1 - d->pad;
    if (d->kh != d->kw) return RGAN_EINVAL;
    g.fgw = FastDiv(d->wout); g.fghw = FastDiv((uint32_t)d->hout * d->wout);
    g.fC = FastDiv(d->cin); g.fKW = FastDiv(d->kw);
    g.out = make_out(d->hout, d->wout, 1, d->ys[0], d->ys[2], d->ys[3], 1, 1, d->cout, 0, 0, d->ys[1]);
    set_pack(p, w, wscale, g.K, g.N, d->cin, d->kw, d->cout, 1, (long long)d->cout * KK, KK, d->kw, 1,
             d->kh, d->kw, 1, 0);
  } else {
    return RGAN_EINVAL;
  }
  p.av = vec_img_ok(g.a);
  p.bv = g.N % 4 == 0;
  choose_tiling(p);
  set_fast(p, d->batch);
  return 0;
}

// data gradient: input dy (cout, hout, wout) -> dx (cin, hin, win)
static int plan_dgrad(const RganConv* d, const float* dy, const float* w, const float* wscale,
                      float* dx, Plan& p) {
  if (!desc_ok(d)) return RGAN_EINVAL;
  GemmArgs& g = p.g;
  const int KK = d->kh * d->kw;
  // Conv2d k4 s2 p1 dgrad == ConvT of dy with W[co][ci] read as [in=co][out=ci]
  if (!d->transposed && is_k4s2p1(d) && d->hin == 2 * d->hout && d->win == 2 * d->wout &&
      plan_narrow_t(p, d->batch, dy, d->ys, d->hout, d->wout, d->cout, w, (long long)d->cin * 16, 16, d->cin, dx,
                    d->xs, wscale, nullptr, RGAN_ACT_NONE, 0.f))
    return 0;
  if (plan_dense1(p, d, 1, nullptr, w, wscale, nullptr, const_cast<float*>(dy), dx, RGAN_ACT_NONE, 0.f)) return 0;
  // ConvT k4 s2 p1 with <= 4 outputs (G's image layer): its dgrad is a Conv2d over the
  // image with <= 4 input channels, W[ci][co] read as [out=ci][in=co] -- the narrow-in kernel
  if (d->transposed && is_k4s2p1(d) && d->hout == 2 * d->hin && d->wout == 2 * d->win) {
    RganConv c = *d;
    c.transposed = 0;
    c.cin = d->cout; c.hin = d->hout; c.win = d->wout;
    c.cout = d->cin; c.hout = d->hin; c.wout = d->win;
    for (int i = 0; i < 4; ++i) { c.xs[i] = d->ys[i]; c.ys[i] = d->xs[i]; }
    if (plan_narrow_in(p, &c, dy, w, wscale, nullptr, dx, RGAN_ACT_NONE, 0.f)) return 0;
  }
  // 3x3 stride-1 Conv2d with <= 4 inputs (arch 1's input layer): its data gradient is the conv
  // of dy with the kernel transposed and flipped (pad 2 - p), <= 4 outputs: the narrow-out
  // kernel, W[co][ci][t] read as [out = ci][in = co][8 - t].  (The mirror case -- <= 4 dy
  // channels into the narrow-in MFMA tile with a 3x3 kernel -- measured no faster than the
  // generic GEMM at C4: 21 vs 19 us per call.)
  if (!d->transposed && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->cin <= 4 &&
      plan_narrow3_out(p, d->batch, dy, d->ys, d->hout, d->wout, d->cout, w, 9, (long long)d->cin * 9, 1, d->cin, dx,
                       d->xs, d->hin, d->win, 2 - d->pad, wscale, nullptr, RGAN_ACT_NONE, 0.f))
    return 0;
  g.a = make_img(dy, d->hout, d->wout, d->cout, d->ys);
  g.C = dx; g.bias = nullptr; g.act = RGAN_ACT_NONE; g.alpha = 0.f;
  g.out = make_out(d->hin, d->win, 1, d->xs[0], d->xs[2], d->xs[3], 1, 1, d->cin, 0, 0, d->xs[1]);
  if (!d->transposed) {
    if (is_k4s2p1(d) && d->hin == 2 * d->hout && d->win == 2 * d->wout) {
      p.mode = MODE_CONVT2;
      p.phases = 4;
      g.M = d->batch * d->hout * d->wout; g.N = d->cin; g.K = 4 * d->cout;
      g.KH = 4; g.KW = 4; g.stride = 2; g.pad = 1;
      g.fgw = FastDiv(d->wout); g.fghw = FastDiv((uint32_t)d->hout * d->wout);
      g.fC = FastDiv(d->cout); g.fKW = FastDiv(2);
      g.out = make_out(d->hout, d->wout, 2, d->xs[0], d->xs[2], d->xs[3], 1, 1, d->cin, 0, 0, d->xs[1]);
      // W[co][ci][kh][kw] read as a ConvT weight [in=co][out=ci]
      set_pack(p, w, wscale, g.K, g.N, d->cout, 2, d->cin, 1, (long long)d->cin * 16, 16, 4, 1, 4, 4, 0, 1);
    } else if (d->stride == 1 && d->kh == d->kw) {
      p.mode = MODE_CONV;
      g.M = d->batch * d->hin * d->win; g.N = d->cin; g.K = KK * d->cout;
      g.KH = d->kh; g.KW = d->kw; g.stride = 1; g.pad = d->kh - 1 - d->pad;
      g.fgw = FastDiv(d->win); g.fghw = FastDiv((uint32_t)d->hin * d->win);
      g.fC = FastDiv(d->cout); g.fKW = FastDiv(d->kw);
      // Wp[(kh,kw,co)][ci] = W[co][ci][k-1-kh][k-1-kw]
      set_pack(p, w, wscale, g.K, g.N, d->cout, d->kw, d->cin, 1, (long long)d->cin * KK, KK, d->kw, 1,
               d->kh, d->kw, 1, 0);
    } else {
      return RGAN_EINVAL;
    }
  } else {
    // transposed conv's dgrad is the direct conv (same k, s, p) with W[ci][co] as [out=ci][in=co]
    p.mode = MODE_CONV;
    g.M = d->batch * d->hin * d->win; g.N = d->cin; g.K = KK * d->cout;
    g.KH = d->kh; g.KW = d->kw; g.stride = d->stride; g.pad = d->pad;
    g.fgw = FastDiv(d->win); g.fghw = FastDiv((uint32_t)d->hin * d->win);
    g.fC = FastDiv(d->cout); g.fKW = FastDiv(d->kw);
    set_pack(p, w, wscale, g.K, g.N, d->cout, d->kw, d->cin, 1, KK, (long long)d->cout * KK, d->kw, 1,
             d->kh, d->kw, 0, 0);
  }
  p.av = vec_img_ok(g.a);
  p.bv = g.N % 4 == 0;
  choose_tiling(p);
  set_fast(p, d->batch);
  return 0;
}

// weight gradient, written in torch weight layout
static int plan_wgrad(const RganConv* d, const float* x, const float* dy, float* dw, Plan& p) {
  if (!desc_ok(d)) return RGAN_EINVAL;
  if (plan_dense1(p, d, 2, x, nullptr, nullptr, nullptr, const_cast<float*>(dy), dw, RGAN_ACT_NONE, 0.f)) return 0;
  if (plan_wgrad3_narrow(p, d, x, dy, dw)) return 0;
  GemmArgs& g = p.g;
  const int KK = d->kh * d->kw;
  p.mode = MODE_WGRAD;
  g.KH = d->kh; g.KW = d->kw; g.stride = d->stride; g.pad = d->pad;
  g.C = dw; g.bias = nullptr; g.act = RGAN_ACT_NONE; g.alpha = 0.f;
  if (!d->transposed) {
    // C[co][(kh,kw,ci)] = sum_p dy[p][co] * im2col(x)[p][(kh,kw,ci)]
    g.a = make_img(dy, d->hout, d->wout, d->cout, d->ys);
    g.im = make_img(x, d->hin, d->win, d->cin, d->xs);
    g.M = d->cout; g.N = KK * d->cin; g.K = d->batch * d->hout * d->wout;
    g.fgw = FastDiv(d->wout); g.fghw = FastDiv((uint32_t)d->hout * d->wout);
    g.fC = FastDiv(d->cin); g.fKW = FastDiv(d->kw);
    g.out = make_out(1, 1, 1, (long long)d->cin * KK, 0, 0, d->kh, d->kw, d->cin, d->kw, 1, KK);
  } else {
    // ConvT weight [ci][co][kh][kw]: the adjoint conv maps dy (hout) -> x (hin)
    g.a = make_img(x, d->hin, d->win, d->cin, d->xs);
    g.im = make_img(dy, d->hout, d->wout, d->cout, d->ys);
    g.M = d->cin; g.N = KK * d->cout; g.K = d->batch * d->hin * d->win;
    g.fgw = FastDiv(d->win); g.fghw = FastDiv((uint32_t)d->hin * d->win);
    g.fC = FastDiv(d->cout); g.fKW = FastDiv(d->kw);
    g.out = make_out(1, 1, 1, (long long)d->cout * KK, 0, 0, d->kh, d->kw, d->cout, d->kw, 1, KK);
  }
  p.av = g.a.sc == 1 && g.M % 4 == 0 && g.a.sh % 4 == 0 && g.a.sw % 4 == 0 && g.a.sb % 4 == 0 &&
         aligned16(g.a.p);
  p.bv = vec_img_ok(g.im);
  choose_tiling(p);
  set_fast(p, d->batch);
  // unsplit FAST wgrads with 4x4 taps: row-contiguous staging + taps_transpose
  const OutMap& o = g.out;
  if (p.fast && g.splits == 1 && p.cfg == CFG_L && o.fnkw.d == 4 && (uint32_t)g.N == 16 * o.fnc.d &&
      o.th == 4 && o.tw == 1 && o.tc == 16 && o.sb % 4 == 0 && o.fnc.d % 4 == 0) {
    p.tap_stage = true;
    p.tap_floats = (size_t)g.M * g.N;
  }
  return 0;
}

static size_t plan_ws_bytes(const Plan& p) {
  const size_t pack = p.prepacked ? 0 : align_up(p.pack_floats * 4, 256);
  return pack + align_up(p.slab_floats * 4, 256) + align_up(p.tap_floats * 4, 256);
}

// pack kernel of a layout: 0 pack_tiled16, 1 pack_tiled (grid gx x gy), -1 pack_weights
static int pack_kind(const PackArgs& a, int& gx, int& gy) {
  // tiled when n is one weight index and the taps are contiguous in W
  if (a.fnco.d == (uint32_t)a.N && a.fnkw.d == 1 && a.s_kw == 1 && a.s_kh == a.KW && a.KH * a.KW <= 16 &&
      (!a.convt2 || (a.KH == 4 && a.KW == 4))) {
    if (a.KH == 4 && a.KW == 4 && a.fpci.d % PK_I == 0 && a.N % PK_O == 0 && a.s_in % 4 == 0 && a.s_out % 4 == 0 &&
        aligned16(a.W) && aligned16(a.out)) {
      gx = (int)a.fpci.d / PK_I;
      gy = a.N / PK_O;
      return 0;
    }
    gx = ceil_div((int)a.fpci.d, PK_I);
    gy = ceil_div(a.N, PK_O);
    return 1;
  }
  return -1;
}

// pack_t2d applies: k = ci alone, n = (tap, co) over a [K][Cout][KH][KW]-contiguous W
static bool pack_t2d_ok(const PackArgs& a) {
  const int T = a.KH * a.KW;
  return !a.convt2 && !a.flip && a.phases == 1 && a.fpci.d == (uint32_t)a.K && a.fnco.d * T == (uint32_t)a.N &&
         a.fnkw.d == (uint32_t)a.KW && a.s_kw == 1 && a.s_kh == a.KW && a.s_out == T && a.s_in == a.N &&
         a.K % PT_K == 0 && a.N % PT_N == 0 && aligned16(a.W) && aligned16(a.out);
}

static void launch_pack(const PackArgs& a, hipStream_t s) {
  if (pack_t2d_ok(a)) {
    pack_t2d<<<dim3(a.N / PT_N, a.K / PT_K), 256, 0, s>>>(a);
    return;
  }
  int gx, gy;
  const int kind = pack_kind(a, gx, gy);
  if (kind == 0) {
    pack_tiled16<<<dim3(gx, gy), 256, 0, s>>>(a);
    return;
  }
  if (kind == 1) {
    pack_tiled<<<dim3(gx, gy), 256, 0, s>>>(a);
    return;
  }
  const int ny = std::min(a.N, 8192);
  pack_weights<<<dim3(ceil_div(a.K, 256), ny, a.phases), 256, 0, s>>>(a);
}

template <int MODE, int BM, int BN, int WM, int WN>
static void launch_cfg(const Plan& p, dim3 grid, hipStream_t s) {
  if (p.fast) gemm_kernel<MODE, BM, BN, WM, WN, true, true, true><<<grid, 256, 0, s>>>(p.g);
  else if (p.av && p.bv) gemm_kernel<MODE, BM, BN, WM, WN, true, true, false><<<grid, 256, 0, s>>>(p.g);
  else if (p.av) gemm_kernel<MODE, BM, BN, WM, WN, true, false, false><<<grid, 256, 0, s>>>(p.g);
  else if (p.bv) gemm_kernel<MODE, BM, BN, WM, WN, false, true, false><<<grid, 256, 0, s>>>(p.g);
  else gemm_kernel<MODE, BM, BN, WM, WN, false, false, false><<<grid, 256, 0, s>>>(p.g);
}

// FAST 128x128 CONV / CONVT2 GEMMs (fwd + dgrad of Conv and ConvT) on the bf16x6 emulation: opt-in
// by rgan_set_gemm_emulation (read at every launch: a captured graph keeps its kernels)
static bool plan_emu(const Plan& p) {
  return p.fast && p.cfg == CFG_L && (p.mode == MODE_CONV || p.mode == MODE_CONVT2) && emu_bf16x6();
}

template <int MODE>
static void launch_mode(const Plan& p, dim3 grid, hipStream_t s) {
  if constexpr (MODE == MODE_CONV || MODE == MODE_CONVT2) {
    if (p.g.pmode && p.g.splits == 1) {  // post_ok: FAST 128x128 (the post-op in the epilogue)
      if (plan_emu(p)) gemm_post_bf16x6<MODE><<<grid, 256, 0, s>>>(p.g);
      else gemm_post<MODE><<<grid, 256, 0, s>>>(p.g);
      return;
    }
    if (plan_emu(p)) {
      gemm_bf16x6<MODE><<<grid, 256, 0, s>>>(p.g);
      return;
    }
  }
  switch (p.cfg) {
    case CFG_L: launch_cfg<MODE, 128, 128, 2, 2>(p, grid, s); break;
    case CFG_M: launch_cfg<MODE, 128, 64, 2, 2>(p, grid, s); break;
    case CFG_S: launch_cfg<MODE, 64, 64, 2, 2>(p, grid, s); break;
    default: launch_cfg<MODE, 256, 32, 4, 1>(p, grid, s); break;
  }
}


// ---------------------------------------------------------------- live launch timing
// When enabled (rgan_profile_begin), every GEMM launch is bracketed by a pair of HIP
// events on its own stream and tagged with the algorithmic FLOPs of the conv op it
// serves (2*B*Cin*Cout*k*k*pixels, the torch flop-counter convention) and with the
// kernel instantiation, so bench.py can report FLOPs / kernel time per kernel symbol.
struct ProfRec {
  hipEvent_t a, b;
  double flops;
  int kid;
};
static bool g_prof = false;
static std::vector<hipEvent_t> g_pool;
static std::vector<ProfRec> g_recs;
static std::vector<std::string> g_kernel_names;
static double g_cur_flops = 0.0;

constexpr int N_KERNEL_IDS = 74;  // 36 (mode, cfg, av, bv) + 9 FAST (mode, cfg) + 2 narrow + 3 dense + img_in + 2 bf16x6 + 2 post + 2 post bf16x6 + 2 narrow 3x3 + 12 (mode, av, bv) + 3 FAST (mode) of the 64x64 tile

static int kernel_id(int mode, int cfg, bool av, bool bv, bool fast = false) {
  if (cfg == CFG_S && mode <= MODE_WGRAD) {
    kernel_id(MODE_NARROW_T, 0, false, false);  // fills the name table
    return fast ? 71 + mode : 59 + mode * 4 + (av ? 2 : 0) + (bv ? 1 : 0);
  }
  const int id = mode == MODE_NARROW_T ? 45
                 : mode == MODE_NARROW_IN ? 46
                 : mode == MODE_DENSE1 ? 47 + cfg
                 : mode == MODE_NARROW3 ? 57
                 : mode == MODE_NARROW3W ? 58
                 : fast ? 36 + mode * 3 + cfg
                        : ((mode * 3 + cfg) * 2 + (av ? 1 : 0)) * 2 + (bv ? 1 : 0);
  if (g_kernel_names.empty()) {
    g_kernel_names.resize(N_KERNEL_IDS);
    const int bm[3] = {128, 128, 256}, bn[3] = {128, 64, 32}, wmv[3] = {2, 2, 4}, wnv[3] = {2, 2, 1};
    for (int m = 0; m < 3; ++m)
      for (int c = 0; c < 3; ++c)
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) {
            char buf[160];
            snprintf(buf, sizeof(buf), "void rgan::gemm_kernel<%d, %d, %d, %d, %d, %s, %s, false>(rgan::GemmArgs)", m,
                     bm[c], bn[c], wmv[c], wnv[c], a ? "true" : "false", b ? "true" : "false");
            g_kernel_names[((m * 3 + c) * 2 + a) * 2 + b] = buf;
          }
    for (int m = 0; m < 3; ++m)
      for (int c = 0; c < 3; ++c) {
        char buf[160];
        snprintf(buf, sizeof(buf), "void rgan::gemm_kernel<%d, %d, %d, %d, %d, true, true, true>(rgan::GemmArgs)", m,
                 bm[c], bn[c], wmv[c], wnv[c]);
        g_kernel_names[36 + m * 3 + c] = buf;
      }
    g_kernel_names[45] = "void rgan::convt2_narrow_mfma<NC>(rgan::NarrowArgs)";
    g_kernel_names[46] = "void rgan::conv_narrow_in_mfma<CI>(rgan::NarrowArgs)";
    g_kernel_names[47] = "void rgan::dense1_fwd<VEC>(rgan::DenseArgs)";
    g_kernel_names[48] = "void rgan::dense1_dgrad<VEC>(rgan::DenseArgs, rgan::FastDiv)";
    g_kernel_names[49] = "rgan::dense1_wgrad(rgan::DenseArgs)";
    g_kernel_names[50] = "void rgan::conv_img_in<CI, WT, ACT>(rgan::NarrowArgs)";
    g_kernel_names[51] = "void rgan::gemm_bf16x6<0>(rgan::GemmArgs)";
    g_kernel_names[52] = "void rgan::gemm_bf16x6<1>(rgan::GemmArgs)";
    g_kernel_names[53] = "void rgan::gemm_post<0>(rgan::GemmArgs)";
    g_kernel_names[54] = "void rgan::gemm_post<1>(rgan::GemmArgs)";
    g_kernel_names[55] = "void rgan::gemm_post_bf16x6<0>(rgan::GemmArgs)";
    g_kernel_names[56] = "void rgan::gemm_post_bf16x6<1>(rgan::GemmArgs)";
    g_kernel_names[57] = "void rgan::conv3_narrow_out<NC>(rgan::NarrowArgs, int)";
    g_kernel_names[58] = "void rgan::wgrad3_narrow<NC>(rgan::NarrowArgs, int, int)";
    for (int m = 0; m < 3; ++m) {
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
          char buf[160];
          snprintf(buf, sizeof(buf), "void rgan::gemm_kernel<%d, 64, 64, 2, 2, %s, %s, false>(rgan::GemmArgs)", m,
                   a ? "true" : "false", b ? "true" : "false");
          g_kernel_names[59 + m * 4 + a * 2 + b] = buf;
        }
      char buf[160];
      snprintf(buf, sizeof(buf), "void rgan::gemm_kernel<%d, 64, 64, 2, 2, true, true, true>(rgan::GemmArgs)", m);
      g_kernel_names[71 + m] = buf;
    }
  }
  return id;
}

static void launch_pack_plan(Plan& p, float* out, hipStream_t s) {
  if (p.mode == MODE_NARROW_T) {
    const int n = p.na.C * 256;
    pack_narrow<<<ceil_div(n, 256), 256, 0, s>>>(p.pk.W, out, p.na.C, p.na.Cout, p.pn_s_in, p.pn_s_out);
  } else {
    p.pk.out = out;
    launch_pack(p.pk, s);
  }
}

static int run_narrow(Plan& p, const float* packed, hipStream_t s) {
  NarrowArgs a = p.na;
  if (p.mode == MODE_NARROW_T) {
    a.w = packed;
    const int ntiles = a.B * ceil_div(a.H, NM_TR) * ceil_div(a.W, NM_TC);
    const int blocks = std::min(ntiles * a.splits, 512);  // persistent: two resident blocks per CU
    switch (a.Cout) {
      case 1: convt2_narrow_mfma<1><<<blocks, 256, 0, s>>>(a, ntiles); break;
      case 2: convt2_narrow_mfma<2><<<blocks, 256, 0, s>>>(a, ntiles); break;
      case 3: convt2_narrow_mfma<3><<<blocks, 256, 0, s>>>(a, ntiles); break;
      default: convt2_narrow_mfma<4><<<blocks, 256, 0, s>>>(a, ntiles); break;
    }
    if (a.splits > 1) {
      const long long n = (long long)a.B * a.Cout * a.Ho * a.Wo;
      narrow_split_reduce<<<(unsigned)std::min<long long>(ceil_div(n, 256LL), 4096), 256, 0, s>>>(a);
    }
  } else if (p.img_in) {
    // persistent waves (two resident blocks of 4 per CU) loop over the 32-pixel wave tiles
    // (32-channel tiles when the width is not a multiple of 128: D at h = 32, 64)
    const int tiles = a.B * a.Ho * a.Wo / 32;
    const bool wide = a.Cout % 128 == 0;
    const dim3 grid(std::min(ceil_div(tiles, 4), 512), a.Cout / (wide ? 128 : 32));
    const int act_kind = a.act == RGAN_ACT_NONE ? 0
                         : (a.act == RGAN_ACT_RELU || (a.act == RGAN_ACT_LRELU && a.alpha <= 1.f)) ? 1 : 2;
#define RGAN_IMG_A(CC, WW, NN)                                                            \
  switch (act_kind) {                                                                     \
    case 0: conv_img_in<CC, WW, 0, NN><<<grid, 256, 0, s>>>(a, tiles); break;             \
    case 1: conv_img_in<CC, WW, 1, NN><<<grid, 256, 0, s>>>(a, tiles); break;             \
    default: conv_img_in<CC, WW, 2, NN><<<grid, 256, 0, s>>>(a, tiles); break;            \
  }
#define RGAN_IMG(CC, NN)                                                          \
  if (a.Wo == 16) RGAN_IMG_A(CC, 16, NN) else RGAN_IMG_A(CC, 32, NN)
    if (!wide) {  // plan_narrow_in: CI == 3
      RGAN_IMG(3, 1)
    } else {
      switch (a.C) {
        case 1: RGAN_IMG(1, 4) break;
        case 2: RGAN_IMG(2, 4) break;
        default: RGAN_IMG(3, 4) break;
      }
    }
#undef RGAN_IMG
#undef RGAN_IMG_A
  } else {
    // persistent: two resident blocks per CU loop over the M tiles
    dim3 grid(std::min(ceil_div(a.B * a.Ho * a.Wo, 128), 512), ceil_div(a.Cout, 128));
    switch (a.C) {
      case 1: conv_narrow_in_mfma<1><<<grid, 256, 0, s>>>(a); break;
      case 2: conv_narrow_in_mfma<2><<<grid, 256, 0, s>>>(a); break;
      case 3: conv_narrow_in_mfma<3><<<grid, 256, 0, s>>>(a); break;
      default: conv_narrow_in_mfma<4><<<grid, 256, 0, s>>>(a); break;
    }
  }
  return 0;
}

static int run_narrow3(Plan& p, hipStream_t s) {
  NarrowArgs a = p.na;
  if (p.mode == MODE_NARROW3) {
    const long long P = (long long)a.B * a.Ho * a.Wo, PW = 64 / (a.C / 4);
    const int steps = a.rows;
    const unsigned blocks = (unsigned)ceil_div(ceil_div(P, PW * steps), (long long)N3_WAVES);
    switch (a.Cout) {
      case 1: conv3_narrow_out<1><<<blocks, 64 * N3_WAVES, 9 * a.C * 1 * 4, s>>>(a, steps); break;
      case 2: conv3_narrow_out<2><<<blocks, 64 * N3_WAVES, 9 * a.C * 2 * 4, s>>>(a, steps); break;
      case 3: conv3_narrow_out<3><<<blocks, 64 * N3_WAVES, 9 * a.C * 3 * 4, s>>>(a, steps); break;
      default: conv3_narrow_out<4><<<blocks, 64 * N3_WAVES, 9 * a.C * 4 * 4, s>>>(a, steps); break;
    }
    return 0;
  }
  const int threads = ceil_div(9 * (a.C / 4), 64) * 64, R = a.rows;
  const size_t lds = wgrad3_lds_bytes(R, a.Wo, a.C, a.Cout);
  switch (a.Cout) {
    case 1: wgrad3_narrow<1><<<a.chunks, threads, lds, s>>>(a, a.C, R); break;
    case 2: wgrad3_narrow<2><<<a.chunks, threads, lds, s>>>(a, a.C, R); break;
    case 3: wgrad3_narrow<3><<<a.chunks, threads, lds, s>>>(a, a.C, R); break;
    default: wgrad3_narrow<4><<<a.chunks, threads, lds, s>>>(a, a.C, R); break;
  }
  RGAN_CHECK_LAUNCH();
  GemmArgs g = p.g;
  g.slab = a.slab;
  const uint32_t per = (uint32_t)g.M * g.N;
  const FastDiv fd((uint32_t)g.N);
  if (g.splits >= 4 * REDW_LANES && per <= 65536) {
    splitk_reduce_wide<MODE_WGRAD><<<dim3((unsigned)ceil_div((long long)per, REDW_OUT), 1), 256, 0, s>>>(g, fd, per);
  } else {
    splitk_reduce<MODE_WGRAD, RED_ANY><<<dim3(std::min<uint32_t>((per + 255) / 256, 8192), 1), 256, 0, s>>>(g, fd, per);
  }
  return 0;
}

static void run_dense1(const Plan& p, const float* packed, hipStream_t s) {
  DenseArgs a = p.da;
  if (p.dense_op != 2) a.w = packed;
  if (p.dense_op != 2) {
    const float* t = p.dense_op == 0 ? a.x : a.out;
    a.vec = a.xsc == 1 && a.C % 4 == 0 && a.xsb % 4 == 0 && a.xsh % 4 == 0 && a.xsw % 4 == 0 && aligned16(t);
  }
  if (p.dense_op == 0) {
    if (a.vec) dense1_fwd<true><<<a.B, 1024, 0, s>>>(a);
    else dense1_fwd<false><<<a.B, 1024, 0, s>>>(a);
  } else if (p.dense_op == 1) {
    const uint32_t per = a.vec ? a.E / 4 : a.E, total = (uint32_t)a.B * per;
    const unsigned blocks = std::min<uint32_t>((total + 255) / 256, 8192);
    if (a.vec) dense1_dgrad<true><<<blocks, 256, 0, s>>>(a, FastDiv(per));
    else dense1_dgrad<false><<<blocks, 256, 0, s>>>(a, FastDiv(per));
  } else {
    dense1_wgrad<<<ceil_div(a.E, 256), 256, 0, s>>>(a);
  }
}

// The vector epilogue can emit BatchNorm segment moments: 128x128 FAST tiles written whole
// (no split-K slab, no tap staging), column n = output channel, 64-row segments that never
// straddle a phase or one of the caller's batch segments.  Call after vec_out is set.
static bool bn_epilogue_ok(const Plan& p) {
  const GemmArgs& g = p.g;
  if (p.mode != MODE_CONV && p.mode != MODE_CONVT2) return false;
  // the 128 x 128 vector epilogue, or the 64 x 64 tile's scalar epilogue (one segment per tile)
  const bool l_vec = p.fast && p.cfg == CFG_L && g.vec_out;
  const bool s_tile = p.cfg == CFG_S && g.act == RGAN_ACT_NONE;
  if (!(l_vec || s_tile) || g.splits != 1 || p.tap_stage) return false;
  if (g.out.fnc.d != (uint32_t)g.N || g.M % 64 != 0 || p.bn_segs < 1) return false;
  if (p.bn_segs > 1 && (p.phases != 1 || g.M % p.bn_segs != 0 || (g.M / p.bn_segs) % 64 != 0)) return false;
  return true;
}

// The split-K reduce can emit the same segment moments (splitk_reduce_bn): channel-contiguous
// float4 output rows (the RED_VEC shape), n = channel, 64-row segments as above.
static bool red_vec_ok(const Plan& p, bool check_ptr) {
  const GemmArgs& g = p.g;
  const OutMap& o = g.out;
  auto al4 = [](long long v) { return (v & 3) == 0; };
  return p.mode != MODE_WGRAD && o.tc == 1 && o.fnc.d % 4 == 0 && g.N % 4 == 0 && al4(o.th) && al4(o.tw) &&
         al4(o.sb) && al4(o.sh) && al4(o.sw) && (!check_ptr || aligned16(g.C));
}

static bool bn_reduce_ok(const Plan& p, bool check_ptr) {
  const GemmArgs& g = p.g;
  if (p.mode != MODE_CONV && p.mode != MODE_CONVT2) return false;
  if (g.splits <= 1 || p.tap_stage || g.accum || !red_vec_ok(p, check_ptr) || g.N < 4 * REDBN_QB) return false;
  if (g.out.fnc.d != (uint32_t)g.N || g.M % 64 != 0 || p.bn_segs < 1) return false;
  if (p.bn_segs > 1 && (p.phases != 1 || g.M % p.bn_segs != 0 || (g.M / p.bn_segs) % 64 != 0)) return false;
  return true;
}

static long long bn_epilogue_segments(const Plan& p) { return (long long)p.phases * (p.g.M / 64); }

// producer post-op (GemmArgs::pmode): unsplit FAST 128x128 tiles (gemm_post's vector
// epilogue) or split tiles (mode 1: every reduce shape of CONV / CONVT2; mode 2: the BN
// reduce); mode 2 also needs n = channel and 64-row segments that never straddle a phase or
// a batch segment.  Call after vec_out is set.
static bool post_ok(const Plan& p, int mode, int nseg, bool check_ptr) {
  const GemmArgs& g = p.g;
  if (p.mode != MODE_CONV && p.mode != MODE_CONVT2) return false;
  if (p.tap_stage || g.accum || g.bias || g.act != RGAN_ACT_NONE) return false;
  const bool whole = g.splits == 1;  // the epilogue sees whole sums
  if (whole && !(p.fast && p.cfg == CFG_L && g.vec_out)) return false;  // gemm_post's epilogue
  if (mode == 1) return true;
  if (mode != 2 || nseg < 1 || g.out.fnc.d != (uint32_t)g.N || g.M % 64 != 0) return false;
  if (nseg > 1 && (g.M % nseg != 0 || (g.M / nseg) % 64 != 0)) return false;
  if (whole) return p.fast && p.cfg == CFG_L && g.vec_out;
  return red_vec_ok(p, check_ptr) && g.N >= 4 * REDBN_QB;
}

static int run_plan(Plan& p, void* ws, size_t ws_bytes, hipStream_t s) {
  if (ws_bytes < plan_ws_bytes(p)) return RGAN_EINVAL;
  if (p.mode == MODE_NARROW_T || p.mode == MODE_NARROW_IN || p.mode == MODE_DENSE1 || p.mode == MODE_NARROW3 ||
      p.mode == MODE_NARROW3W) {
    const float* packed = p.prepacked;
    if (p.pack && !packed) {
      if (!ws) return RGAN_EINVAL;
      launch_pack_plan(p, (float*)ws, s);
      RGAN_CHECK_LAUNCH();
      packed = (const float*)ws;
    }
    if (p.slab_floats)  // narrow ConvT channel-split partial sums, after the pack
      p.na.slab = (float*)((char*)ws + (p.prepacked ? 0 : align_up(p.pack_floats * 4, 256)));
    ProfRec rec{};
    const bool prof = g_prof && g_recs.size() * 2 + 2 <= g_pool.size();
    if (prof) {
      rec.a = g_pool[g_recs.size() * 2];
      rec.b = g_pool[g_recs.size() * 2 + 1];
      rec.flops = g_cur_flops;
      rec.kid = kernel_id(p.mode, p.mode == MODE_DENSE1 ? p.dense_op : 0, false, false);
      if (p.mode == MODE_NARROW_IN && p.img_in) rec.kid = 50;
      hipEventRecord(rec.a, s);
    }
    if (p.mode == MODE_DENSE1) run_dense1(p, packed, s);
    else if (p.mode == MODE_NARROW3 || p.mode == MODE_NARROW3W) run_narrow3(p, s);
    else run_narrow(p, packed, s);
    RGAN_CHECK_LAUNCH();
    if (prof) {
      hipEventRecord(rec.b, s);
      g_recs.push_back(rec);
    }
    return 0;
  }
  if (p.g.M <= 0 || p.g.N <= 0 || p.g.K <= 0) return RGAN_EINVAL;
  char* w = (char*)ws;
  if (p.pack && p.prepacked) {
    p.g.Bw = p.prepacked;
  } else if (p.pack) {
    if (!ws) return RGAN_EINVAL;
    p.pk.out = (float*)w;
    p.g.Bw = p.pk.out;
    w += align_up(p.pack_floats * 4, 256);
    launch_pack(p.pk, s);
    RGAN_CHECK_LAUNCH();
  }
  p.g.slab = p.slab_floats ? (float*)w : nullptr;
  float* tap_dst = nullptr;
  long long tap_osb = 0;
  if (p.tap_stage && !aligned16(p.g.C)) p.tap_stage = false;  // workspace stays sized for it
  const int accum = p.g.accum;
  if (p.tap_stage) {
    tap_dst = p.g.C;
    tap_osb = p.g.out.sb;
    p.g.accum = 0;  // the staging buffer is written fresh; taps_transpose accumulates
    p.g.C = (float*)(w + align_up(p.slab_floats * 4, 256));
    p.g.out = make_out(1, 1, 1, p.g.N, 0, 0, 1, 1, p.g.N, 0, 0, 1);  // [M][N], n contiguous
  }
  {
    const OutMap& o = p.g.out;
    auto al4 = [](long long v) { return (v & 3) == 0; };
    p.g.vec_out = p.mode != MODE_WGRAD && o.tc == 1 && o.fnc.d % 4 == 0 && p.g.N % 4 == 0 && al4(o.th) &&
                  al4(o.tw) && al4(o.sb) && al4(o.sh) && al4(o.sw) && aligned16(p.g.C);
  }
  p.bn_fused = p.bn_part && (bn_epilogue_ok(p) || bn_reduce_ok(p, true));
  p.g.bnp = p.bn_fused ? p.bn_part : nullptr;
  p.post_fused = p.post && !p.bn_fused && post_ok(p, p.post->mode, p.post->nseg, true) &&
                 (p.post->mode != 2 || bn_epilogue_segments(p) <= p.post->part_segments);
  if (p.post_fused) {
    const RganPost& q = *p.post;
    p.g.pmode = q.mode; p.g.pact = q.act; p.g.palpha = q.alpha; p.g.pnseg = q.nseg;
    p.g.px = q.x; p.g.pst = q.stats; p.g.pgam = q.gamma; p.g.pbet = q.beta; p.g.ppart = q.part;
  } else {
    p.g.pmode = 0;
  }
  int bm, bn;
  tile_dims(p.cfg, bm, bn);
  const int tiles_m = ceil_div(p.g.M, bm);
  p.g.nph = p.phases;
  p.g.xgroup = p.fast && p.mode != MODE_WGRAD && tiles_m % 8 == 0 ? 3 : 0;
  // weight-column grouping where the weights dominate: under A-row grouping every XCD fetches
  // the whole weight (D's 2048 -> 4096 conv at C3: 4.36 GB of FETCH per launch for a 537 MB
  // weight; 1.01 GB grouped by weight columns).  Under weight-column grouping every XCD reads
  // the input through its im2col windows instead, which costs more than the input's bytes: at
  // a 2:1 weight / input ratio (D's 1024 -> 2048 conv) it fetched 2.02 GB against 1.33, hence
  // the factor 4 (run r4g)
  if (p.fast && p.mode != MODE_WGRAD && p.g.tiles_n % 8 == 0 &&
      (long long)p.g.bw_bytes * p.phases > 4LL * p.g.a_bytes && tiles_m * p.phases > 1)
    p.g.xgroup = 2;
  dim3 grid = p.g.xgroup ? dim3(tiles_m * p.g.tiles_n * p.phases, 1, p.g.splits)
                         : dim3(tiles_m * p.g.tiles_n, 1, p.phases * p.g.splits);
  ProfRec rec{};
  const bool prof = g_prof && g_recs.size() * 2 + 2 <= g_pool.size();
  if (prof) {
    rec.a = g_pool[g_recs.size() * 2];
    rec.b = g_pool[g_recs.size() * 2 + 1];
    rec.flops = g_cur_flops;
    rec.kid = kernel_id(p.mode, p.cfg, p.av, p.bv, p.fast);
    if (plan_emu(p)) rec.kid = 51 + p.mode;
    if (p.g.pmode && p.g.splits == 1) rec.kid = (plan_emu(p) ? 55 : 53) + p.mode;
    hipEventRecord(rec.a, s);
  }
  switch (p.mode) {
    case MODE_CONV: launch_mode<MODE_CONV>(p, grid, s); break;
    case MODE_CONVT2: launch_mode<MODE_CONVT2>(p, grid, s); break;
    default: launch_mode<MODE_WGRAD>(p, grid, s); break;
  }
  RGAN_CHECK_LAUNCH();
  if (prof) {
    hipEventRecord(rec.b, s);
    g_recs.push_back(rec);
  }
  p.g.accum = accum;
  if (p.tap_stage) {
    const int cin = p.g.N / 16;
    taps_transpose<<<dim3(ceil_div(cin, 64), p.g.M), 256, 0, s>>>(p.g.C, tap_dst, cin, tap_osb, p.g.accum);
    RGAN_CHECK_LAUNCH();
  }
  if (p.g.splits > 1) {
    const GemmArgs& g = p.g;
    const OutMap& o = g.out;
    auto al4 = [](long long v) { return (v & 3) == 0; };
    int kind = RED_ANY;
    uint32_t per = (uint32_t)g.M * g.N, d = g.N;
    if (p.mode != MODE_WGRAD && o.tc == 1 && o.fnc.d % 4 == 0 && g.N % 4 == 0 && al4(o.th) &&
        al4(o.tw) && al4(o.sb) && al4(o.sh) && al4(o.sw) && ((uintptr_t)g.C & 15) == 0) {
      kind = RED_VEC;
      per /= 4;
      d = g.N / 4;
    } else if (p.mode == MODE_WGRAD && o.fnkw.d == 4 && (uint32_t)g.N == 16 * o.fnc.d && o.th == 4 &&
               o.tw == 1 && o.tc == 16 && al4(o.sb) && ((uintptr_t)g.C & 15) == 0) {
      kind = RED_TAPS;
      per /= 4;
      d = o.fnc.d;
    }
    if (p.bn_fused || g.pmode == 2) {  // the RED_VEC shape with segment moments / backward sums
      const int Q = g.N / 4;
      int qb = 1;  // quads per block: 8 (32 channels, 128-B row pieces), fewer for narrow N
      while (qb * 2 <= std::min(Q, REDBN_QB)) qb *= 2;
      const dim3 bgrid((unsigned)((g.M / 64) * ceil_div(Q, qb)), p.phases);
      if (g.pmode == 2) splitk_reduce_bn<true><<<bgrid, 256, 0, s>>>(g, p.mode == MODE_CONVT2, qb);
      else splitk_reduce_bn<false><<<bgrid, 256, 0, s>>>(g, p.mode == MODE_CONVT2, qb);
      RGAN_CHECK_LAUNCH();
      return 0;
    }
    const FastDiv fd(d);
    if (kind == RED_ANY && g.splits >= 4 * REDW_LANES && per <= 65536) {  // few outputs, long chains
      const dim3 wgrid((unsigned)ceil_div((long long)per, REDW_OUT), p.phases);
      switch (p.mode) {
        case MODE_CONV: splitk_reduce_wide<MODE_CONV><<<wgrid, 256, 0, s>>>(g, fd, per); break;
        case MODE_CONVT2: splitk_reduce_wide<MODE_CONVT2><<<wgrid, 256, 0, s>>>(g, fd, per); break;
        default: splitk_reduce_wide<MODE_WGRAD><<<wgrid, 256, 0, s>>>(g, fd, per); break;
      }
      RGAN_CHECK_LAUNCH();
      return 0;
    }
    const dim3 rgrid((unsigned)std::min<uint32_t>((per + 255) / 256, 8192), p.phases);
#define RGAN_RED(MD)                                                                   \
  switch (kind) {                                                                      \
    case RED_VEC: splitk_reduce<MD, RED_VEC><<<rgrid, 256, 0, s>>>(g, fd, per); break;  \
    case RED_TAPS: splitk_reduce<MD, RED_TAPS><<<rgrid, 256, 0, s>>>(g, fd, per); break; \
    default: splitk_reduce<MD, RED_ANY><<<rgrid, 256, 0, s>>>(g, fd, per); break;       \
  }
    switch (p.mode) {
      case MODE_CONV: RGAN_RED(MODE_CONV) break;
      case MODE_CONVT2: RGAN_RED(MODE_CONVT2) break;
      default: RGAN_RED(MODE_WGRAD) break;
    }
#undef RGAN_RED
    RGAN_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace rgan

using namespace rgan;

extern "C" size_t rgan_conv_workspace(const RganConv* d, int which, int prepacked) {
  Plan p;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  int rc;
  if (which == 0) rc = plan_fwd(d, dummy, dummy, nullptr, nullptr, (float*)dummy, 0, 0.f, p);
  else if (which == 1) rc = plan_dgrad(d, dummy, dummy, nullptr, (float*)dummy, p);
  else rc = plan_wgrad(d, dummy, dummy, (float*)dummy, p);
  if (rc) return 0;
  if (prepacked && which != 2) p.prepacked = dummy;
  size_t extra = 0;
  if (which == 2)  // bias-gradient reduction scratch (rgan_channel_sum, or the fused per-split sums), after the plan's
    extra = align_up(std::max(rgan_bn_partial_bytes((long long)d->batch * d->hout * d->wout, d->cout),
                              (size_t)p.g.splits * p.g.M * sizeof(double) + 256), 256);
  return align_up(plan_ws_bytes(p), 256) + extra + 256;  // never 0 for a valid descriptor
}

extern "C" size_t rgan_conv_pack_floats(const RganConv* d, int which) {
  Plan p;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  int rc = which == 0 ? plan_fwd(d, dummy, dummy, nullptr, nullptr, (float*)dummy, 0, 0.f, p)
                      : plan_dgrad(d, dummy, dummy, nullptr, (float*)dummy, p);
  if (rc || which > 1 || !p.pack) return 0;  // 0: no packed layout (or unsupported)
  return p.pack_floats;
}

extern "C" int rgan_conv_pack(const RganConv* d, int which, const float* w, float* packed, void* stream) {
  if (!w || !packed || which < 0 || which > 1) return RGAN_EINVAL;
  Plan p;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  int rc = which == 0 ? plan_fwd(d, dummy, w, nullptr, nullptr, (float*)dummy, 0, 0.f, p)
                      : plan_dgrad(d, dummy, w, nullptr, (float*)dummy, p);
  if (rc) return rc;
  if (!p.pack) return RGAN_EINVAL;
  launch_pack_plan(p, packed, (hipStream_t)stream);
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_conv_pack_batch(int n, const RganConv* const* d, const int* which, const float* const* w,
                                    float* const* packed, void* stream) {
  if (n < 0 || (n > 0 && (!d || !which || !w || !packed))) return RGAN_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  PackBatch b{};
  long long blocks = 0;
  auto flush = [&]() {
    if (b.n == 0) return;
    b.first[b.n] = (int)blocks;
    pack_multi<<<(unsigned)blocks, 256, 0, s>>>(b);
    b = PackBatch{};
    blocks = 0;
  };
  for (int i = 0; i < n; ++i) {
    if (!w[i] || !packed[i] || which[i] < 0 || which[i] > 1) return RGAN_EINVAL;
    Plan p;
    const int rc = which[i] == 0 ? plan_fwd(d[i], dummy, w[i], nullptr, nullptr, (float*)dummy, 0, 0.f, p)
                                 : plan_dgrad(d[i], dummy, w[i], nullptr, (float*)dummy, p);
    if (rc) return rc;
    if (!p.pack) return RGAN_EINVAL;
    int gx = 0, gy = 0;
    const int kind = p.mode == MODE_NARROW_T ? -1 : (p.pk.out = packed[i], pack_kind(p.pk, gx, gy));
    if (kind < 0) {  // narrow / generic layouts: their own launch
      launch_pack_plan(p, packed[i], s);
      RGAN_CHECK_LAUNCH();
      continue;
    }
    if (b.n == PACK_BATCH || blocks + (long long)gx * gy >= (1LL << 30)) flush();
    b.a[b.n] = p.pk;
    b.kind[b.n] = kind;
    b.gx[b.n] = gx;
    b.first[b.n] = (int)blocks;
    blocks += (long long)gx * gy;
    ++b.n;
  }
  flush();
  RGAN_CHECK_LAUNCH();
  return 0;
}

extern "C" int rgan_adam_step_inc(float* step, void* stream);

extern "C" int rgan_adam_packed(int ntensors, float* const* params, const float* const* grads,
                                float* const* exp_avg, float* const* exp_avg_sq, const long long* numel,
                                const double* hyper, float* step, int npacks, const RganAdamPack* packs,
                                void* stream) {
  RGAN_REQUIRE(ntensors >= 0 && npacks >= 0 && hyper && step && (npacks == 0 || packs));
  RGAN_REQUIRE(ntensors == 0 || (params && grads && exp_avg && exp_avg_sq && numel));
  hipStream_t s = (hipStream_t)stream;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  for (int j = 0; j < ntensors; ++j)
    RGAN_REQUIRE(params[j] && grads[j] && exp_avg[j] && exp_avg_sq[j] && numel[j] >= 0 && numel[j] < (1LL << 31));
  // plan every layout: in-kernel (AdamPackT) or a repack launch after the step
  std::vector<std::vector<AdamPackT>> per(ntensors);
  std::vector<Plan> later;
  std::vector<float*> later_out;
  for (int i = 0; i < npacks; ++i) {
    const RganAdamPack& q = packs[i];
    RGAN_REQUIRE(q.d && q.packed && q.tensor >= 0 && q.tensor < ntensors && (q.which == 0 || q.which == 1));
    Plan p;
    const float* W = params[q.tensor];
    const int rc = q.which == 0 ? plan_fwd(q.d, dummy, W, nullptr, nullptr, (float*)dummy, 0, 0.f, p)
                                : plan_dgrad(q.d, dummy, W, nullptr, (float*)dummy, p);
    if (rc) return rc;
    RGAN_REQUIRE(p.pack);
    const long long n = numel[q.tensor];
    AdamPackT t{};
    t.out = q.packed;
    bool ok = false;
    const PackArgs& a = p.pk;
    if (p.mode == MODE_NARROW_T) {
      const int C = p.na.C, NC = p.na.Cout;
      ok = p.pn_s_out == 16 && p.pn_s_in == 16LL * NC && (long long)C * NC * 16 == n;
      t.kind = APK_NARROW; t.A = C; t.B = NC; t.KK = 16;
    } else if (pack_t2d_ok(a)) {
      const int T = a.KH * a.KW, Cout = (int)a.fnco.d;
      ok = (long long)a.K * Cout * T == n;
      t.kind = APK_T2D; t.A = a.K; t.B = Cout; t.KK = T; t.K = a.K;
      t.in_is_a = 1;  // k = ci = the weight's first index: runs of 4 consecutive ci
    } else {
      int gx, gy;
      const int kind = pack_kind(a, gx, gy);
      const int KK = a.KH * a.KW, Nin = (int)a.fpci.d, Nout = a.N;
      if (kind >= 0 && a.s_kw == 1 && a.s_kh == a.KW && (long long)Nin * Nout * KK == n) {
        t.kind = APK_TILED; t.KK = KK; t.KW = a.KW; t.flip = a.flip; t.convt2 = a.convt2;
        t.Nin = Nin; t.Nout = Nout; t.K = a.K;
        if (a.s_in == KK && a.s_out == (long long)Nin * KK) {         // in = second index
          ok = true; t.in_is_a = 0; t.A = Nout; t.B = Nin;
        } else if (a.s_out == KK && a.s_in == (long long)Nout * KK) {  // in = first index
          ok = true; t.in_is_a = 1; t.A = Nin; t.B = Nout;
        }
      }
    }
    if (ok) {
      per[q.tensor].push_back(t);
    } else {
      later.push_back(p);
      later_out.push_back(q.packed);
    }
  }
  RGAN_CHECK_LAUNCH();
  AdamPackBatch b{};
  long long blocks = 0;
  int np = 0;
  bool bumped = false;
  auto flush = [&](bool last) -> int {
    if (b.cnt == 0) return 0;
    b.first[b.cnt] = (int)blocks;
    if (blocks > 0) {
      adam_pack_kernel<<<(unsigned)blocks, AP_THREADS, 0, s>>>(b, hyper, step, last ? 1 : 0);
      bumped = last;
    }
    RGAN_CHECK_LAUNCH();
    b = AdamPackBatch{};
    blocks = 0;
    np = 0;
    return 0;
  };
  for (int j = 0; j < ntensors; ++j) {
    auto& L = per[j];
    const int nt = (int)L.size();
    RGAN_REQUIRE(nt <= AP_MAXP);
    if (b.cnt == AP_MAXT || np + nt > AP_MAXP) {
      const int rc = flush(false);
      if (rc) return rc;
    }
    AdamPackTensor X{params[j], grads[j], exp_avg[j], exp_avg_sq[j], numel[j], 0, 0, np, nt};
    bool brick = nt > 0 && ((((uintptr_t)params[j] | (uintptr_t)grads[j] | (uintptr_t)exp_avg[j] |
                               (uintptr_t)exp_avg_sq[j]) & 15) == 0);
    for (const auto& t : L) {
      brick = brick && (t.kind == APK_TILED || t.kind == APK_T2D) && t.KK == 16 && t.A == L[0].A &&
              t.B == L[0].B && t.A % 32 == 0 && t.B % 32 == 0 && aligned16(t.out);
      b.pk[np++] = t;
    }
    X.brick = brick;
    X.bricks_b = brick ? L[0].B / 32 : 0;
    const long long nb = brick ? (long long)(L[0].A / 32) * (L[0].B / 32) : (numel[j] + AP_FLAT - 1) / AP_FLAT;
    b.t[b.cnt] = X;
    b.first[b.cnt] = (int)blocks;
    blocks += nb;
    RGAN_REQUIRE(blocks < (1LL << 30));
    ++b.cnt;
  }
  int rc = flush(true);
  if (rc) return rc;
  if (!bumped) {  // no block ran the last launch's ticket: a separate increment
    rc = rgan_adam_step_inc(step, stream);
    if (rc) return rc;
  }
  for (size_t i = 0; i < later.size(); ++i) {  // layouts the kernel does not write: repack
    launch_pack_plan(later[i], later_out[i], s);
    RGAN_CHECK_LAUNCH();
  }
  return 0;
}

static double conv_flops(const RganConv* d) {
  if (!d) return 0.0;  // (the planner refuses it next)
  const double pix = d->transposed ? (double)d->hin * d->win : (double)d->hout * d->wout;
  return 2.0 * d->batch * (double)d->cin * d->cout * d->kh * d->kw * pix;
}

extern "C" int rgan_conv_fwd(const RganConv* d, const float* x, const float* w, const float* wpacked,
                             const float* wscale, const float* bias, float* y, int act, float act_alpha, void* ws,
                             size_t ws_bytes, void* stream) {
  RGAN_REQUIRE(act_ok(act));
  if (!x || (!w && !wpacked) || !y) return RGAN_EINVAL;
  g_cur_flops = conv_flops(d);
  Plan p;
  int rc = plan_fwd(d, x, w, wscale, bias, y, act, act_alpha, p);
  if (rc) return rc;
  if (!p.pack && !w) return RGAN_EINVAL;  // kernels that read the torch layout
  p.prepacked = wpacked;
  return run_plan(p, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" long long rgan_conv_bn_segments(const RganConv* d, int segs) {
  Plan p;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  if (segs < 1 || plan_fwd(d, dummy, dummy, nullptr, nullptr, (float*)dummy, 0, 0.f, p)) return 0;
  if (p.mode != MODE_CONV && p.mode != MODE_CONVT2) return 0;
  const OutMap& o = p.g.out;
  auto al4 = [](long long v) { return (v & 3) == 0; };
  p.g.vec_out = o.tc == 1 && o.fnc.d % 4 == 0 && p.g.N % 4 == 0 && al4(o.th) && al4(o.tw) && al4(o.sb) &&
                al4(o.sh) && al4(o.sw);
  p.bn_segs = segs;
  return (bn_epilogue_ok(p) || bn_reduce_ok(p, false)) ? bn_epilogue_segments(p) : 0;
}

extern "C" int rgan_conv_fwd_bn(const RganConv* d, const float* x, const float* w, const float* wpacked,
                                const float* wscale, const float* bias, float* y, void* ws, size_t ws_bytes,
                                double* bn_part, long long part_segments, int segs, int* fused, void* stream) {
  if (!x || (!w && !wpacked) || !y || !fused || segs < 1) return RGAN_EINVAL;
  *fused = 0;
  g_cur_flops = conv_flops(d);
  Plan p;
  int rc = plan_fwd(d, x, w, wscale, bias, y, 0, 0.f, p);
  if (rc) return rc;
  if (!p.pack && !w) return RGAN_EINVAL;
  p.prepacked = wpacked;
  const bool want = bn_part && p.mode != MODE_NARROW_T && p.mode != MODE_NARROW_IN && p.mode != MODE_DENSE1 &&
                    bn_epilogue_segments(p) <= part_segments;
  p.bn_part = want ? bn_part : nullptr;
  p.bn_segs = segs;
  rc = run_plan(p, ws, ws_bytes, (hipStream_t)stream);
  if (rc) return rc;
  *fused = p.bn_fused ? 1 : 0;
  return 0;
}

extern "C" int rgan_conv_dgrad(const RganConv* d, const float* dy, const float* w, const float* wpacked,
                               const float* wscale, float* dx, void* ws, size_t ws_bytes, void* stream) {
  if (!dy || (!w && !wpacked) || !dx) return RGAN_EINVAL;
  g_cur_flops = conv_flops(d);
  Plan p;
  int rc = plan_dgrad(d, dy, w, wscale, dx, p);
  if (rc) return rc;
  if (!p.pack && !w) return RGAN_EINVAL;  // kernels that read the torch layout
  p.prepacked = wpacked;
  return run_plan(p, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" long long rgan_conv_post_segments(const RganConv* d, int which, int mode, int nseg, int* phases) {
  Plan p;
  alignas(16) static const float dummy[4] = {0, 0, 0, 0};
  int rc = which == 0 ? plan_fwd(d, dummy, dummy, nullptr, nullptr, (float*)dummy, 0, 0.f, p)
                      : plan_dgrad(d, dummy, dummy, nullptr, (float*)dummy, p);
  if (rc || (which != 0 && which != 1) || mode != 2) return 0;
  const OutMap& o = p.g.out;
  auto al4 = [](long long v) { return (v & 3) == 0; };
  p.g.vec_out = p.mode != MODE_WGRAD && o.tc == 1 && o.fnc.d % 4 == 0 && p.g.N % 4 == 0 && al4(o.th) &&
                al4(o.tw) && al4(o.sb) && al4(o.sh) && al4(o.sw);
  if (phases) *phases = p.phases;
  return post_ok(p, mode, nseg, false) ? bn_epilogue_segments(p) : 0;
}

extern "C" int rgan_conv_post(const RganConv* d, int which, const float* in, const float* w, const float* wpacked,
                              const float* wscale, float* out, void* ws, size_t ws_bytes, const RganPost* post,
                              int* fused, void* stream) {
  if (!in || (!w && !wpacked) || !out || !fused || !post || (which != 0 && which != 1)) return RGAN_EINVAL;
  if (!post->x || (post->mode != 1 && post->mode != 2) || !act_ok(post->act)) return RGAN_EINVAL;
  if (post->mode == 2 && (!post->stats || !post->part || post->nseg < 1)) return RGAN_EINVAL;
  *fused = 0;
  g_cur_flops = conv_flops(d);
  Plan p;
  int rc = which == 0 ? plan_fwd(d, in, w, wscale, nullptr, out, RGAN_ACT_NONE, 0.f, p)
                      : plan_dgrad(d, in, w, wscale, out, p);
  if (rc) return rc;
  if (!p.pack && !w) return RGAN_EINVAL;
  p.prepacked = wpacked;
  p.post = post;
  rc = run_plan(p, ws, ws_bytes, (hipStream_t)stream);
  if (rc) return rc;
  *fused = p.post_fused ? 1 : 0;
  return 0;
}

extern "C" int rgan_conv_wgrad(const RganConv* d, const float* x, const float* dy, float* dw,
                               float* dbias, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return rgan_conv_wgrad_rows(d, x, dy, dw, dbias, 0, accumulate, ws, ws_bytes, stream);
}

extern "C" int rgan_conv_wgrad_rows(const RganConv* d, const float* x, const float* dy, float* dw, float* dbias,
                                    long long dbias_row0, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !dy || !dw) return RGAN_EINVAL;
  g_cur_flops = conv_flops(d);
  Plan p;
  int rc = plan_wgrad(d, x, dy, dw, p);
  if (rc) return rc;
  p.g.accum = accumulate ? 1 : 0;
  p.da.accum = p.g.accum;
  const size_t plan_bytes = align_up(plan_ws_bytes(p), 256);
  // per-output-channel sum of dy over pixel rows [dbias_row0, P) (Conv2d and ConvTranspose2d
  // alike: dy has cout channels), checked before anything is launched
  const long long P = (long long)d->batch * d->hout * d->wout;
  long long sp = 0;
  if (dbias) {
    if (dbias_row0 < 0 || dbias_row0 >= P) return RGAN_EINVAL;
    if ((long long)d->hout * d->wout == 1) {
      sp = d->ys[0];
    } else {
      if (d->ys[1] != 1 || d->ys[3] != d->cout || d->ys[2] != (long long)d->wout * d->cout ||
          d->ys[0] != (long long)d->hout * d->wout * d->cout)
        return RGAN_EINVAL;
      sp = d->cout;
    }
    const size_t need = plan_bytes + rgan_bn_partial_bytes(P - dbias_row0, d->cout);
    if (!ws || ws_bytes < need) return RGAN_EINVAL;
  }
  // a FAST Conv2d weight gradient stages dy as its A operand: the GEMM sums the bias
  // gradient from those tiles (GemmArgs::dbias, from the BK-aligned pixel row db_k0 on)
  // instead of a channel-sum pass over dy
  const bool bias_fused = dbias && p.mode == MODE_WGRAD && p.fast && !d->transposed && ws_bytes >= plan_bytes &&
                          dbias_row0 % BK == 0 && dbias_row0 <= (long long)INT32_MAX &&
                          (p.g.splits == 1 || (size_t)p.g.splits * p.g.M * sizeof(double) <= ws_bytes - plan_bytes);
  if (bias_fused) {
    p.g.dbias = dbias;
    p.g.db_accum = accumulate ? 1 : 0;
    p.g.db_k0 = (int)dbias_row0;
    p.g.dbp = p.g.splits > 1 ? reinterpret_cast<double*>((char*)ws + plan_bytes) : nullptr;
  }
  rc = run_plan(p, ws, ws_bytes, (hipStream_t)stream);
  if (rc) return rc;
  if (dbias && !bias_fused)
    return rgan_channel_sum(dy + dbias_row0 * sp, P - dbias_row0, d->cout, sp, d->ys[1], dbias, accumulate,
                            (char*)ws + plan_bytes, stream);
  return 0;
}

extern "C" int rgan_set_gemm_emulation(int on) {
  if (on != 0 && on != 1) return -1;
  const int prev = emu_bf16x6() ? 1 : 0;
  g_emu.store(on, std::memory_order_relaxed);
  return prev;
}

extern "C" int rgan_profile_begin(int capacity) {
  if (capacity <= 0) return RGAN_EINVAL;
  for (auto e : g_pool) hipEventDestroy(e);
  g_pool.clear();
  g_recs.clear();
  g_pool.resize((size_t)capacity * 2);
  for (auto& e : g_pool) {
    hipError_t rc = hipEventCreate(&e);
    if (rc != hipSuccess) return (int)rc;
  }
  g_prof = true;
  return 0;
}

// Stops recording, waits for the last event and returns totals over all recorded GEMM
// launches; per-kernel-symbol totals are then available via rgan_profile_kernel.
static std::vector<double> g_kms, g_kflops;
static std::vector<long long> g_kn;

extern "C" int rgan_profile_end(double* total_ms, double* total_flops, long long* launches) {
  g_prof = false;
  g_kms.assign(N_KERNEL_IDS, 0.0);
  g_kflops.assign(N_KERNEL_IDS, 0.0);
  g_kn.assign(N_KERNEL_IDS, 0);
  double ms = 0.0, fl = 0.0;
  if (!g_recs.empty()) {
    hipError_t rc = hipEventSynchronize(g_recs.back().b);
    if (rc != hipSuccess) return (int)rc;
  }
  for (const ProfRec& r : g_recs) {
    float t = 0.f;
    hipError_t rc = hipEventElapsedTime(&t, r.a, r.b);
    if (rc != hipSuccess) return (int)rc;
    ms += t;
    fl += r.flops;
    g_kms[r.kid] += t;
    g_kflops[r.kid] += r.flops;
    g_kn[r.kid] += 1;
  }
  if (total_ms) *total_ms = ms;
  if (total_flops) *total_flops = fl;
  if (launches) *launches = (long long)g_recs.size();
  g_recs.clear();
  return 0;
}

extern "C" int rgan_profile_kernel(int idx, char* name, int name_len, double* ms, double* flops, long long* n) {
  if (idx < 0 || idx >= N_KERNEL_IDS || g_kms.empty()) return RGAN_EINVAL;
  kernel_id(0, 0, false, false);
  if (name && name_len > 0) snprintf(name, name_len, "%s", g_kernel_names[idx].c_str());
  if (ms) *ms = g_kms[idx];
  if (flops) *flops = g_kflops[idx];
  if (n) *n = g_kn[idx];
  return 0;
}
