// pkc_rnn_persist.hip — persistent time loops of a block-sparse liGRU layer in bf16 step mode
// (north_star: "recurrent time-step loops fused per wavefront"; the per-step form of the same
// arithmetic is pkc_rnn_impl.h rnn_fwd_mm / rnn_bwd_mm + rnn_bwd_epi).
//
// Reference: liGRU neural_networks.py:1573-1584 (z = sig(wz + Uz h); hc = act(wh + Uh h) * drop;
// h = z h + (1 - z) hc), both directions as one 2B-row batch (:1536-1538).  The recurrence couples
// the units of a row, never two rows: row r's h_t needs only row r's h_{t-1}.  So the whole T-step
// loop of a layer runs as ONE launch of ceil(B2 / RPW) workgroups, each owning RPW rows for every
// step, with no cross-workgroup hand-off at all:
//   * the layer's nonzero U blocks (C3's HCGS masks keep ~175 of the 648 blocks of 16 units x 32
//     k per gate) are loaded ONCE: the first NFR fragments of each wave as registers (B operands
//     of v_mfma_f32_16x16x32_bf16), the rest into LDS;
//   * h_{t-1} of the workgroup's rows is the A operand, a bf16 image in LDS (double-buffered by
//     step parity) whose batch rows sit at MFMA rows 0, 4, 8, 12, so the C layout (row 4 q + i in
//     lane group q) puts batch row q's result in register 0 of lane group q: every lane carries a
//     live element out of the chain;
//   * per step: each wave runs its fragment list (the fragments dealt to the waves in equal runs
//     by the host; a tile cut between two waves flushes its second part into a spill-over tile),
//     storing each finished tile's products to LDS, with the next slot's operands read under the
//     current slot's MFMAs; barrier; the cell update spread over all threads (adding a cut tile's
//     spill-over; gates / h / y stores, the next A image); barrier.  (LDS float atomics for the
//     cut tiles measured 2x slower steps than these plain stores.)
// The per-step form pays a launch boundary and a cross-XCD fetch of h_{t-1} every step (~5 us for
// C3); here a step is the MFMA chains, two LDS passes and two workgroup barriers.
// The BPTT loop is the same with U^T fragments (output tile = 16 columns k, contraction = units j
// of both gates summed in one chain) and the dgates_t images as A operands: dh_{t-1} =
// sum_g dgates_g U_g, then the liGRU gate gradients of step t-1 (gate_grads / bwd_step_epi).
// Numerics: the bf16 step mode's (bf16 h / dgates / U operands, fp32 accumulation and cell math);
// only the order of the fp32 block sums differs from the per-step kernels.
//
// Plan tables (host, pkc.engine.persist_plans): per wave NF int32 entries, bits 0-7 output tile,
// 8-15 block + 1, bit 16 flush (the last fragment of this wave's part of the tile), bit 17 valid,
// bit 18 the flush of a cut tile's second part, 19-21 its spill-over tile.
#define PKC_RNN_PERSIST
#include "pkc_rnn_impl.h"

namespace pkc {
namespace persist {

constexpr int NW = 8, NT = 64 * NW;     // two waves per SIMD
// batch rows per workgroup (1, 2 or 4): the fragment loop is the same for any RPW (every workgroup
// multiplies all of the layer's U blocks), the cell update and its stores scale with it — one row
// per workgroup puts B2 workgroups on the loop, each with a quarter of the 4-row form's update
constexpr int RPW = 1;
static_assert(RPW == 1 || RPW == 2 || RPW == 4, "rows per workgroup: 1, 2 or 4");
constexpr int RSH = RPW == 4 ? 2 : (RPW == 2 ? 3 : 4);   // MFMA row c -> batch row c >> RSH
// fragment slots per wave (plan width: ceil(fragments / 8) <= NF, C3: 22) and how many of them
// are register-resident (the rest, NF - NFR per wave, in LDS); 16 register slots leave room for
// the one-slot operand look-ahead
constexpr int FNF = 23, FNFR = 15;
constexpr int BNF = 22, BNFR = 14;
constexpr int HMAX = 576;               // H <= HMAX (36 tiles of 16)
// row stride of the bf16 A images (elements): 16-byte rows at dword offsets 0, 48, 32, 16 mod 64
// banks for the 4 live rows, so an A-fragment read (4 rows x 4 lane groups x 16 B) is conflict-free
constexpr int HP = 608;
constexpr int IMG = RPW * HP;           // one A image (bf16 elements)
// the cell update works on pairs of adjacent units (H is even): 8-byte loads and stores, 4-byte
// bf16 pairs — half the memory instructions of one element per lane
constexpr int PPT = (RPW * HMAX / 2 + NT - 1) / NT;   // epilogue unit pairs per thread
constexpr int EPT = 2 * PPT;                          // epilogue elements per thread
constexpr int FRAG = 64 * 16;           // bytes of one B fragment (64 lanes x 8 bf16)

typedef __attribute__((ext_vector_type(8))) __bf16 bf8;
typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
typedef __attribute__((ext_vector_type(2))) float fl2;

__device__ __forceinline__ bf8 zero8() {
  bf8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
  return v;
}

// 8 bf16 of a row at k0 .. k0+7 (zero past kmax / when !ok); rows of even length: 4-byte pairs
__device__ __forceinline__ bf8 load8(const __bf16* row, bool ok, int k0, int kmax) {
  bf8 v;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const bool in = ok && k0 + j < kmax;
    const bf2 x = *reinterpret_cast<const bf2*>(row + (in ? k0 + j : 0));
    v[j] = in ? x[0] : (__bf16)0.f;
    v[j + 1] = in ? x[1] : (__bf16)0.f;
  }
  return v;
}

// A fragment of 32-wide block kb: lane (MFMA row c, lane group q) holds k = 32 kb + 8 q .. + 7 of
// batch row c >> RSH (RPW = 4: MFMA rows 4 i .. 4 i + 3 all carry batch row i); only row 4 q of
// each result (register 0 of lane group q, batch row (4 q) >> RSH) is used, the duplicates are
// ignored — so every lane reads
// (same-address lanes are LDS broadcasts) and the fragment loop stays branch-free: the compiler
// can issue the next fragments' LDS reads under the current MFMAs
__device__ __forceinline__ bf8 a_frag(const __bf16* img, int c, int q, int kb) {
  return *reinterpret_cast<const bf8*>(img + (c >> RSH) * HP + 32 * kb + 8 * q);
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also drains every outstanding global
// load and store of the thread (vmcnt), which would stall each step on the previous step's output
// stores and this step's prefetched pre-activations; the loop exchanges data through LDS alone
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Phase trace (PKC_TRACE measurement builds only): wave `lane 0` of workgroup 0 accumulates the
// shader-clock cycles of each step phase over the loop — 0 fragment loop, 1 wait at the products
// barrier, 2 cell-update values, 3 store issue, 4 wait at the step-end barrier — read back with
// pkc_trace_read_persist ([fwd, bwd][wave][8]: the five sums, then T).  The stamps sit where the
// loop already drains the LDS counter.
#ifdef PKC_TRACE
__device__ unsigned long long ptrace_buf[2 * NW * 8];
#define PTR_DECL unsigned long long pt_acc[5] = {0, 0, 0, 0, 0}, pt_last = 0
#define PTR_MARK(i)                                                     \
  do {                                                                  \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();       \
    if ((i) > 0) pt_acc[(i) - 1] += now_ - pt_last;                     \
    pt_last = now_;                                                     \
  } while (0)
#define PTR_STORE(k)                                                    \
  do {                                                                  \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {                   \
      volatile unsigned long long* b_ = ptrace_buf + ((k) * NW + (threadIdx.x >> 6)) * 8; \
      for (int i_ = 0; i_ < 5; ++i_) b_[i_] = pt_acc[i_];               \
      b_[5] = (unsigned long long)T;                                    \
    }                                                                   \
  } while (0)
#else
#define PTR_DECL do { } while (0)
#define PTR_MARK(i) do { } while (0)
#define PTR_STORE(k) do { } while (0)
#endif

__device__ __forceinline__ int pl_tile(int e) { return e & 255; }
__device__ __forceinline__ int pl_blk(int e) { return ((e >> 8) & 255) - 1; }
__device__ __forceinline__ bool pl_flush(int e) { return (e >> 16) & 1; }
__device__ __forceinline__ bool pl_valid(int e) { return (e >> 17) & 1; }
__device__ __forceinline__ bool pl_spill(int e) { return (e >> 18) & 1; }
__device__ __forceinline__ int pl_sidx(int e) { return (e >> 19) & 7; }
constexpr int NTILE = HMAX / 16;        // output tiles of a layer
// product-tile row: H columns, 16 for tile columns past H, then NW spill-over tiles of 16
constexpr int XCOL = HMAX + 16, AW = XCOL + NW * 16;
// static LDS of the two loops against gfx950's 160 KiB per workgroup (the BPTT sits
// within 1.6 KB of it; any growth must fail here, not as a link error of the whole library)
constexpr int LDS_LIMIT = 160 * 1024;
constexpr int FWD_LDS = NW * (FNF - FNFR) * 2 * FRAG + IMG * 2 + 2 * RPW * AW * 4 + NTILE * 4;
constexpr int BWD_LDS = NW * (BNF - BNFR) * 2 * FRAG + 2 * 2 * IMG * 2 + RPW * AW * 4 + NTILE * 4;
static_assert(FWD_LDS <= LDS_LIMIT, "persistent forward loop: static LDS over 160 KiB");
static_assert(BWD_LDS <= LDS_LIMIT, "persistent BPTT loop: static LDS over 160 KiB");
// el: an element's A-image position (bits 0-15) and its tile's spill-over index + 1 (bits 16-19)
__device__ __forceinline__ int el_pos(int el) { return el & 0xFFFF; }
__device__ __forceinline__ int el_spill(int el) { return (el >> 16) - 1; }
// the slot's 32-wide A block (block 0 for an empty slot: any block, its B fragments are zeros)
__device__ __forceinline__ int slot_blk(int e) { return pl_valid(e) ? max(pl_blk(e), 0) : 0; }

// A cell-update element's offsets, from its A-image position el (row rl = el / HP, unit u) — an
// unused slot (el < 0) takes element 0 of the workgroup's first row (valid addresses, unused
// values).  Recomputed where used (a few integer ops) rather than held in registers through the
// fragment loop: the opaque copy keeps the compiler from hoisting them out of the time loop.
struct ElemOff {
  int ost;    // (t, r, u) of (T, B2, H): + t B2 H
  int opre;   // (tt, rr, u) of (T, B, H): + tt B H
  int oout;   // (tt, rr, u) of (T, B, D): + tt B D
  bool rev;   // the reversed direction (rows >= B): time T-1-t
};
__device__ __forceinline__ ElemOff elem_off(int el, int r0, int H, int B, int D, bool bidir) {
  int e = el < 0 ? 0 : el_pos(el);
  asm volatile("" : "+v"(e));
  const int rl = e / HP, u = e - rl * HP, r = r0 + rl;
  ElemOff o;
  o.rev = bidir && r >= B;
  const int rr = o.rev ? r - B : r;
  o.ost = r * H + u;
  o.opre = rr * H + u;
  o.oout = rr * D + (o.rev ? H : 0) + u;
  return o;
}

// The B fragments of one wave's plan: slots < NFR into registers, the rest into the wave's LDS
// region (lane-linear 16-byte pieces: conflict-free reads).  src(g, tile, c) = the row of U_h (fwd:
// unit row, k contiguous) or U^T (bwd: k row, j contiguous) that lane column c reads.
template <int NF, int NFR>
struct Frags {
  static constexpr int NFL = NF - NFR;
  bf8 r[NFR][2];
  // slot f, gate g: registers (f < NFR; f is a compile-time index after unrolling) or LDS
  __device__ __forceinline__ void put(char* ufl, int w, int lane, int f, int g, const bf8& v) {
    if (f < NFR) r[f < NFR ? f : 0][g] = v;
    else *reinterpret_cast<bf8*>(ufl + ((w * NFL + (f - NFR)) * 2 + g) * FRAG + 16 * lane) = v;
  }
  __device__ __forceinline__ bf8 get(const char* ufl, int w, int lane, int f, int g) const {
    if (f < NFR) return r[f < NFR ? f : 0][g];
    return *reinterpret_cast<const bf8*>(ufl + ((w * NFL + (f - NFR)) * 2 + g) * FRAG + 16 * lane);
  }
};

// ----------------------------------------------------------------------------------- forward
__global__ __launch_bounds__(NT) void fwd_loop(pkc_rnn_args a) {
  constexpr int NF = FNF, NFR = FNFR;
  using Fr = Frags<NF, NFR>;
  __shared__ __attribute__((aligned(16))) char ufl[NW * Fr::NFL * 2 * FRAG];   // LDS fragments
  // A: h_{t-1}, one image: the cell update rewrites it after the products barrier (every read of
  // the step is done) and the next step reads it after the step-end barrier
  __shared__ __attribute__((aligned(16))) __bf16 hl[IMG];
  __shared__ float accl[2][RPW][AW];            // the step's products (see AW)
  __shared__ int tspill[NTILE];                  // tile -> its spill-over tile (-1: not cut)
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int r0 = blockIdx.x * RPW, nr = min(RPW, B2 - r0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int64_t TBH = (int64_t)T * a.B * H, TB2H = (int64_t)T * B2 * H;
  for (int i = tid; i < IMG / 2; i += NT) reinterpret_cast<uint32_t*>(hl)[i] = 0u;
  int pl[NF];
  Fr fr;
#pragma clang loop unroll(full)
  for (int f = 0; f < NF; ++f) {
    const int e = __builtin_amdgcn_readfirstlane(a.persist_fwd[w * NF + f]);
    pl[f] = e;
    const int kb = pl_valid(e) ? pl_blk(e) : -1;
    const int unit = pl_tile(e) * 16 + c;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const __bf16* row = reinterpret_cast<const __bf16*>(a.U_h[g]) + (int64_t)(unit < H ? unit : 0) * H;
      fr.put(ufl, w, lane, f, g, kb >= 0 ? load8(row, unit < H, 32 * kb + 8 * q, H) : zero8());
    }
  }
  // this thread's cell-update elements: the same every step (h_{t-1} and the mask in registers);
  // 32-bit element offsets (every saved tensor of a layer holds < 2^31 elements: host check) so the
  // stores take a uniform base + per-lane offset
  const int B = a.B, D = ix.bidir ? 2 * H : H;
  // tiles without a fragment keep zero products; the spill-over map from the plans
  for (int i = tid; i < 2 * RPW * AW; i += NT) (&accl[0][0][0])[i] = 0.f;
  for (int i = tid; i < NTILE; i += NT) tspill[i] = -1;
  __syncthreads();
  if (lane == 0)
    for (int f = 0; f < NF; ++f)
      if (pl_valid(pl[f]) && pl_flush(pl[f]) && pl_spill(pl[f])) tspill[pl_tile(pl[f])] = pl_sidx(pl[f]);
  __syncthreads();
  int el[PPT];                                    // per pair: its first unit (see el_pos)
  float hp[EPT], mk[EPT];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int e = 2 * (tid + NT * j);              // the pair's first element (u even)
    const bool ok = e < nr * H;
    const int rl = ok ? e / H : 0, u = ok ? e % H : 0, r = r0 + rl;
    // the pair in the A image and its tile's spill-over (-1: none)
    el[j] = ok ? (rl * HP + u) | ((tspill[u >> 4] + 1) << 16) : -1;
    hp[2 * j] = hp[2 * j + 1] = 0.f;               // h_init = 0
    mk[2 * j] = ok ? drop_val(a, r, u, B2) : 0.f;
    mk[2 * j + 1] = ok ? drop_val(a, r, u + 1, B2) : 0.f;
  }
  const float* __restrict__ wpre = a.wpre;
  float* __restrict__ gates = a.gates;
  float* __restrict__ hs = a.hs;
  __bf16* __restrict__ hs_h = reinterpret_cast<__bf16*>(a.hs_h);
  float* __restrict__ y = a.y;
  const int BH = B * H, B2H = B2 * H, BD = B * D, iTBH = (int)TBH;
  PTR_DECL;
  for (int t = 0; t < T; ++t) {
    PTR_MARK(0);
    const __bf16* img = hl;
    // this step's gate pre-activations (independent of the recurrence: in flight during the MFMAs)
    // (every lane loads — element 0 for an unused slot — and every lane consumes the values below:
    // a load under a per-lane branch leaves its register pending on the other path, and the next
    // step's overwrite would wait for every outstanding memory operation, this step's stores too)
    fl2 wz[PPT], wh[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const ElemOff o = elem_off(el[j], r0, H, B, D, ix.bidir);
      const int pi = el[j] >= 0 ? (o.rev ? T - 1 - t : t) * BH + o.opre : 0;   // even
      wz[j] = *reinterpret_cast<const fl2*>(wpre + pi);
      wh[j] = *reinterpret_cast<const fl2*>(wpre + iTBH + pi);
    }
    f32x4 az = {0.f, 0.f, 0.f, 0.f}, ah = {0.f, 0.f, 0.f, 0.f};
    // straight-line over the plan (empty slots multiply zero B fragments); slot f + 1's operands
    // (the A fragment, and B from LDS past the register slots) are read before slot f's MFMAs, so
    // their LDS latency overlaps the chain
    // (A fragments two slots ahead: they are the reads every slot makes)
    bf8 av = a_frag(img, c, q, slot_blk(pl[0])), av1 = a_frag(img, c, q, slot_blk(pl[NF > 1 ? 1 : 0]));
    bf8 bz = fr.get(ufl, w, lane, 0, 0), bh = fr.get(ufl, w, lane, 0, 1);
#pragma clang loop unroll(full)
    for (int f = 0; f < NF; ++f) {
      const int e = pl[f];
      const int fn = f + 1 < NF ? f + 1 : f, fn2 = f + 2 < NF ? f + 2 : f;
      const bf8 an2 = a_frag(img, c, q, slot_blk(pl[fn2]));
      const bf8 bzn = fr.get(ufl, w, lane, fn, 0), bhn = fr.get(ufl, w, lane, fn, 1);
      az = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bz, az, 0, 0, 0);
      ah = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bh, ah, 0, 0, 0);
      av = av1;
      av1 = an2;
      bz = bzn;
      bh = bhn;
      const bool fl = pl_valid(e) && pl_flush(e);
      const int unit = pl_tile(e) * 16 + c;
      // batch row q, unit: register 0; a cut tile's second part to its spill-over tile
      const int col = pl_spill(e) ? XCOL + 16 * pl_sidx(e) + c : (unit < H ? unit : HMAX + c);
      if (fl) {
        accl[0][(4 * q) >> RSH][col] = az[0];   // (RPW < 4: lane groups of one row write
        accl[1][(4 * q) >> RSH][col] = ah[0];   // the same value)
      }
      const f32x4 zero = {0.f, 0.f, 0.f, 0.f};       // restart after a flush (a select: a
      az = fl ? zero : az;                            // multiply by 0 would turn inf into NaN)
      ah = fl ? zero : ah;
      // one slot per scheduling window: the look-ahead above is the overlap, and no later slot's
      // reads are hoisted here (4 VGPRs each)
      __builtin_amdgcn_sched_barrier(0);
    }
    PTR_MARK(1);
    lds_barrier();
    PTR_MARK(2);
    // liGRU cell update (pkc_rnn_impl.h fwd_epi, CELL_LIGRU)
    __bf16* nimg = hl;
    const int tst = t * B2H;
    // every element's values first, then the stores: vmcnt is one in-order counter for loads and
    // stores alike, so a load consumed after this step's first stores would wait for those too
    fl2 zv[PPT], hv[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const bool ok = el[j] >= 0;
      const int e = ok ? el_pos(el[j]) : 0;
      const int rl = e / HP, u = e - rl * HP;
      const int sp = ok ? el_spill(el[j]) : -1, xc = XCOL + 16 * (sp < 0 ? 0 : sp) + (u & 15);
      const fl2 xz = *reinterpret_cast<const fl2*>(&accl[0][rl][xc]);    // (selects, no branch)
      const fl2 xh = *reinterpret_cast<const fl2*>(&accl[1][rl][xc]);
      const fl2 pz = *reinterpret_cast<const fl2*>(&accl[0][rl][u]);
      const fl2 ph = *reinterpret_cast<const fl2*>(&accl[1][rl][u]);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int k = 2 * j + i;
        zv[j][i] = sigm_fast(wz[j][i] + (pz[i] + (sp < 0 ? 0.f : xz[i])));   // (bf16 mode)
        hv[j][i] = act_fwd(a.act, wh[j][i] + (ph[i] + (sp < 0 ? 0.f : xh[i])));
        const float h = zv[j][i] * hp[k] + (1.f - zv[j][i]) * (hv[j][i] * mk[k]);
        hp[k] = ok ? h : 0.f;                        // (a select: consumed on every lane)
      }
    }
    PTR_MARK(3);
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      if (el[j] < 0) continue;
      const ElemOff o = elem_off(el[j], r0, H, B, D, ix.bidir);
      const int si = tst + o.ost;                    // even: every offset below is
      const fl2 h2 = {hp[2 * j], hp[2 * j + 1]};
      const bf2 hb = {(__bf16)h2[0], (__bf16)h2[1]};
      *reinterpret_cast<fl2*>(gates + si) = zv[j];
      *reinterpret_cast<fl2*>(gates + (int)TB2H + si) = hv[j];
      *reinterpret_cast<fl2*>(hs + si + B2H) = h2;   // hs[t + 1]
      *reinterpret_cast<bf2*>(hs_h + si + B2H) = hb;
      *reinterpret_cast<fl2*>(y + (o.rev ? T - 1 - t : t) * BD + o.oout) = h2;
      *reinterpret_cast<bf2*>(nimg + el_pos(el[j])) = hb;
    }
    PTR_MARK(4);
    lds_barrier();
    PTR_MARK(5);
  }
  PTR_STORE(0);
}

// ----------------------------------------------------------------------------------- BPTT
template <bool DY2>                     // DY2: dL/dy in two slabs (one: the common case)
__global__ __launch_bounds__(NT) void bwd_loop(pkc_rnn_args a) {
  constexpr int NF = BNF, NFR = BNFR;
  using Fr = Frags<NF, NFR>;
  __shared__ __attribute__((aligned(16))) char ufl[NW * Fr::NFL * 2 * FRAG];
  __shared__ __attribute__((aligned(16))) __bf16 dl[2][2 * IMG];    // [step parity][gate z, h]
  __shared__ float accl[RPW][AW];               // dh products of the step (see AW)
  __shared__ int tspill[NTILE];                  // tile -> its spill-over tile (-1: not cut)
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int r0 = blockIdx.x * RPW, nr = min(RPW, B2 - r0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int64_t TB2H = (int64_t)T * B2 * H;
  const int64_t n = (int64_t)B2 * H;
  for (int i = tid; i < 2 * IMG; i += NT) reinterpret_cast<uint32_t*>(&dl[0][0])[i] = 0u;
  // U^T fragments: B[j][k] = U[j][k] with column k = 16 tile + c, rows j = 32 jb + 8 q .. + 7,
  // contiguous in ut_h[g][k][j]
  int pl[NF];
  Fr fr;
#pragma clang loop unroll(full)
  for (int f = 0; f < NF; ++f) {
    const int e = __builtin_amdgcn_readfirstlane(a.persist_bwd[w * NF + f]);
    pl[f] = e;
    const int jb = pl_valid(e) ? pl_blk(e) : -1;
    const int k = pl_tile(e) * 16 + c;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const __bf16* row = reinterpret_cast<const __bf16*>(a.ut_h) + (int64_t)g * H * H +
                          (int64_t)(k < H ? k : 0) * H;
      fr.put(ufl, w, lane, f, g, jb >= 0 ? load8(row, k < H, 32 * jb + 8 * q, H) : zero8());
    }
  }
  const int B = a.B, D = ix.bidir ? 2 * H : H, BD = B * D;
  // per element: its A-image position (elem_off gives the offsets where they are used); an unused
  // slot reads element 0 of the workgroup's first row: every lane's addresses without a select
  // or branch in the step loop
  for (int i = tid; i < RPW * AW; i += NT) (&accl[0][0])[i] = 0.f;   // tiles without fragments
  for (int i = tid; i < NTILE; i += NT) tspill[i] = -1;
  __syncthreads();
  if (lane == 0)
    for (int f = 0; f < NF; ++f)
      if (pl_valid(pl[f]) && pl_flush(pl[f]) && pl_spill(pl[f])) tspill[pl_tile(pl[f])] = pl_sidx(pl[f]);
  __syncthreads();
  int el[PPT];                                   // per unit pair (as the forward's)
  float gc[EPT], mk[EPT];
  const __bf16* dgh_in = reinterpret_cast<const __bf16*>(a.dgates_h);
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int e = 2 * (tid + NT * j);
    const bool ok = e < nr * H;
    const int rl = ok ? e / H : 0, k = ok ? e % H : 0, r = r0 + rl;
    el[j] = ok ? (rl * HP + k) | ((tspill[k >> 4] + 1) << 16) : -1;
    const int ostj = r * H + k;
    // step T-1 (rnn_bwd_init): g_{T-1} in carry slot (T-1-(T-1)) & 1 = 0, and its dgates (bf16)
    // as the first A images
    const fl2 g2 = *reinterpret_cast<const fl2*>(a.work + ostj);
    gc[2 * j] = ok ? g2[0] : 0.f;
    gc[2 * j + 1] = ok ? g2[1] : 0.f;
    mk[2 * j] = ok ? drop_val(a, r, k, B2) : 0.f;
    mk[2 * j + 1] = ok ? drop_val(a, r, k + 1, B2) : 0.f;
    if (ok) {
      const int si = (T - 1) * B2 * H + ostj;
      const int par = (T - 1) & 1;
      *reinterpret_cast<bf2*>(&dl[par][el_pos(el[j])]) = *reinterpret_cast<const bf2*>(dgh_in + si);
      *reinterpret_cast<bf2*>(&dl[par][IMG + el_pos(el[j])]) =
          *reinterpret_cast<const bf2*>(dgh_in + (int)TB2H + si);
    }
  }
  const float* __restrict__ gates = a.gates;
  const float* __restrict__ hs = a.hs;
  const float* __restrict__ dy = a.dy;
  float* __restrict__ dgates = a.dgates;
  __bf16* __restrict__ dgh = reinterpret_cast<__bf16*>(a.dgates_h);
  const int B2H = B2 * H, iTB2H = (int)TB2H;
  const int dys = DY2 ? (int)a.dy_slab_stride : 0;   // < 2^31 (rnn_persist_ok)
  float zc[EPT];                                // z_{tt+1}, carried from the step before
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const fl2 z2 = *reinterpret_cast<const fl2*>(
        gates + (T - 1) * B2H + elem_off(el[j], r0, H, B, D, ix.bidir).ost);
    zc[2 * j] = z2[0];
    zc[2 * j + 1] = z2[1];
  }
  __syncthreads();
  PTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    PTR_MARK(0);
    const int t = tt + 1;
    const __bf16* img = dl[t & 1];
    const int tst = tt * B2H;
    fl2 dyv[PPT], hpv[PPT], ztt[PPT], hct[PPT];
    // (unconditional loads and uses, as the forward's; every offset is even)
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const ElemOff o = elem_off(el[j], r0, H, B, D, ix.bidir);
      const int si = tst + o.ost;
      const int oi = (o.rev ? T - 1 - tt : tt) * BD + o.oout;
      // one or two slabs (rnn_persist_ok; the engine sums more beforehand)
      const fl2 d0 = *reinterpret_cast<const fl2*>(dy + oi);
      dyv[j] = DY2 ? d0 + *reinterpret_cast<const fl2*>(dy + dys + oi) : d0;
      hpv[j] = *reinterpret_cast<const fl2*>(hs + si);     // h_{tt-1} = hs[tt]
      ztt[j] = *reinterpret_cast<const fl2*>(gates + si);
      hct[j] = *reinterpret_cast<const fl2*>(gates + iTB2H + si);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // operand look-ahead by half a slot (the BPTT holds more per-element state than the forward
    // and has two A images): gate 1's operands of slot f are read under gate 0's MFMA, gate 0's of
    // slot f + 1 under gate 1's
    bf8 a0 = a_frag(img, c, q, slot_blk(pl[0])), b0 = fr.get(ufl, w, lane, 0, 0);
#pragma clang loop unroll(full)
    for (int f = 0; f < NF; ++f) {
      const int e = pl[f];
      const int fn = f + 1 < NF ? f + 1 : f;
      const bf8 a1 = a_frag(img + IMG, c, q, slot_blk(e)), b1 = fr.get(ufl, w, lane, f, 1);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
      const bf8 a0n = a_frag(img, c, q, slot_blk(pl[fn])), b0n = fr.get(ufl, w, lane, fn, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
      a0 = a0n;
      b0 = b0n;
      const bool fl = pl_valid(e) && pl_flush(e);
      const int k = pl_tile(e) * 16 + c;
      if (fl)   // (a cut tile's second part to its spill-over tile)
        accl[(4 * q) >> RSH][pl_spill(e) ? XCOL + 16 * pl_sidx(e) + c : (k < H ? k : HMAX + c)] = acc[0];
      acc = fl ? f32x4{0.f, 0.f, 0.f, 0.f} : acc;
      __builtin_amdgcn_sched_barrier(0);
    }
    PTR_MARK(1);
    lds_barrier();
    PTR_MARK(2);
    // bwd_step_epi + gate_grads (CELL_LIGRU) for step tt
    __bf16* nimg = dl[tt & 1];
    // values first, then the stores (as the forward's)
    fl2 d0v[PPT], d1v[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const bool ok = el[j] >= 0;
      const int e = ok ? el_pos(el[j]) : 0;
      const int rl = e / HP, k = e - rl * HP;
      const int sp = ok ? el_spill(el[j]) : -1;
      const fl2 xd = *reinterpret_cast<const fl2*>(&accl[rl][XCOL + 16 * (sp < 0 ? 0 : sp) + (k & 15)]);
      const fl2 pd = *reinterpret_cast<const fl2*>(&accl[rl][k]);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kk = 2 * j + i;
        const float dh = (pd[i] + (sp < 0 ? 0.f : xd[i])) + gc[kk] * zc[kk];   // z_{tt+1}: previous
        const float g = dyv[j][i] + dh;
        const float z = ztt[j][i], hcr = hct[j][i], m = mk[kk];
        const float hc = hcr * m;
        const float dz = g * (hpv[j][i] - hc);
        const float dhc = g * (1.f - z);
        d0v[j][i] = dz * z * (1.f - z);
        d1v[j][i] = dhc * m * act_bwd_out(a.act, hcr);
        gc[kk] = ok ? g : 0.f;                        // (a select: consumed on every lane)
        zc[kk] = z;
      }
      // the next step's A images on every lane (an unused slot writes columns HP - 2, HP - 1 of
      // row 0, padding no fragment reads): the values are consumed here, ahead of the stores
      const int ei = ok ? e : HP - 2;
      *reinterpret_cast<bf2*>(nimg + ei) = bf2{(__bf16)d0v[j][0], (__bf16)d0v[j][1]};
      *reinterpret_cast<bf2*>(nimg + IMG + ei) = bf2{(__bf16)d1v[j][0], (__bf16)d1v[j][1]};
    }
    PTR_MARK(3);
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      if (el[j] < 0) continue;
      const int si = tst + elem_off(el[j], r0, H, B, D, ix.bidir).ost;
      *reinterpret_cast<fl2*>(dgates + si) = d0v[j];
      *reinterpret_cast<fl2*>(dgates + iTB2H + si) = d1v[j];
      *reinterpret_cast<bf2*>(dgh + si) = bf2{(__bf16)d0v[j][0], (__bf16)d0v[j][1]};
      *reinterpret_cast<bf2*>(dgh + iTB2H + si) = bf2{(__bf16)d1v[j][0], (__bf16)d1v[j][1]};
    }
    PTR_MARK(4);
    lds_barrier();
    PTR_MARK(5);
  }
  PTR_STORE(1);
  // the carry of step 0 where the per-step form leaves it (slot (T-1) & 1)
  if (T > 1) {
    const int p0 = (T - 1) & 1;
#pragma unroll
    for (int j = 0; j < PPT; ++j)
      if (el[j] >= 0)
        *reinterpret_cast<fl2*>(a.work + p0 * n + elem_off(el[j], r0, H, B, D, ix.bidir).ost) =
            fl2{gc[2 * j], gc[2 * j + 1]};
  }
}

}  // namespace persist

bool rnn_persist_ok(const pkc_rnn_args* a, bool bwd) {
  using namespace persist;
  const int64_t B2 = a->bidir ? 2 * a->B : a->B;
  const int64_t D = a->bidir ? 2 * a->H : a->H;
  if (2 * (int64_t)a->T * B2 * a->H >= (1ll << 31) || (int64_t)a->T * a->B * D >= (1ll << 31))
    return false;                               // 32-bit element offsets
  if (bwd && (a->dy_nslab > 2 || (a->dy_nslab == 2 && 2 * a->dy_slab_stride >= (1ll << 31))))
    return false;                               // dL/dy: at most 2 slabs, 32-bit offsets
  return a->cell == PKC_CELL_LIGRU && a->step_bf16 && (bwd ? a->persist_bwd : a->persist_fwd) &&
         a->persist_kb == FNF && a->H <= HMAX && a->H % 2 == 0 && !a->ln_gamma && a->qbits <= 0 &&
         a->hs_h && a->U_h[0] && a->U_h[1] && (!bwd || (a->ut_h && a->dgates_h));
}

int rnn_persist_fwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace persist;
  const int B2 = a->bidir ? 2 * a->B : a->B;
  hipLaunchKernelGGL(fwd_loop, dim3((B2 + RPW - 1) / RPW), dim3(NT), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_fwd persistent loop");
  return PKC_OK;
}

int rnn_persist_bwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace persist;
  const int B2 = a->bidir ? 2 * a->B : a->B;
  if (a->dy_nslab > 1)
    hipLaunchKernelGGL(bwd_loop<true>, dim3((B2 + RPW - 1) / RPW), dim3(NT), 0, s, *a);
  else
    hipLaunchKernelGGL(bwd_loop<false>, dim3((B2 + RPW - 1) / RPW), dim3(NT), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd persistent loop");
  return PKC_OK;
}

}  // namespace pkc

// plan-table geometry for the host (pkc.engine builds the per-wave fragment lists)
extern "C" int pkc_rnn_persist_geometry(int* nwaves, int* nslots_fwd, int* nslots_bwd,
                                        int* rows_per_wg, int* hmax) {
  using namespace pkc::persist;
  if (nwaves) *nwaves = NW;
  if (nslots_fwd) *nslots_fwd = FNF;
  if (nslots_bwd) *nslots_bwd = BNF;
  if (rows_per_wg) *rows_per_wg = RPW;
  if (hmax) *hmax = HMAX;
  return PKC_OK;
}

#ifdef PKC_TRACE
// measurement builds only: the persistent loops' per-wave phase sums (n <= 2 * 8 * 8)
extern "C" int pkc_trace_read_persist(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pkc::persist::ptrace_buf),
                             sizeof(unsigned long long) * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
