// prl_ppo_split.h — the HEAD-SPLIT latency form of the persistent update engine (included by
// prl_ppo_update.hip inside namespace prl, after the engine's helpers; PPO/PPO.py:216-255).
//
// The two-head (discrete) nets — CartPole, the headline's C2 at the reference's mini_batch 512 —
// have an actor head and a critic head that share only the trunk:
//     logp  = actor(trunk(x)),  V = critic(trunk(x)),  loss = surrogate(logp) + 0.5 SmoothL1(V)
// so the actor's loss gradient never needs the critic's outputs and vice versa, and the trunk's
// gradient is the SUM of what each head sends back through it (GroupNorm's backward is linear in
// the incoming gradient for fixed forward statistics).  This form gives each head its own
// workgroup: a tile group of 16 rows is two workgroups on two CUs, role 0 (trunk + actor head)
// and role 1 (trunk + critic head), each 4 waves = one wave per SIMD, wave w = channel block w.
// Against the 8-wave kernel (both heads on one CU, two waves per SIMD sharing the matrix pipe
// and the VALU issue slots), a SIMD issues one head's MFMAs and GroupNorm / loss VALU instead
// of two, and each workgroup's AdamW updates only the parameters its tile reads (trunk + own
// head: ~53 % of the image) — the other head's image entries go stale in its LDS, unread.
//
// The step:
//   phase A  role r runs its 16-row tile (3 workgroup barriers) into an LDS gradient image and
//            publishes its head's quads into part[gt] and its trunk quads (+ its loss-partial
//            quad) into part[gt] (role 0) or part2[gt] (role 1) — sc1 16-B stores, drained;
//            arrival on counter A (G = 2 Gt workgroups);
//   phase B  slice owner g (of G) sums its quads over the Gt partials of part, and for the trunk
//            and loss quads also over the Gt of part2, in a fixed order with float64
//            accumulators; publishes the slice (sc1), counter B;
//   phase C  every workgroup loads the whole reduced gradient and forms clip_grad_norm_'s norm
//            in ONE canonical order (thread t: quads t + 256 i; the same DPP tree; waves in
//            order) — the same bits on both roles, so the trunk copies the two roles update stay
//            bit-identical — then AdamW on its owned quads only.
// Hand-offs are the engine's (Guideline 16 first row: sc1 payload, drained, one arriving lane
// behind a barrier, sc1 polls; sharded counters).  The trunk gradient is summed in another
// order than the 8-wave kernel's (per head, then across heads in float64), so the two forms
// agree to float32 rounding, not bit for bit (tests/test_engine_gpu.py::test_split_*).

// SPL_NW waves run the tile (wave w = channel block w); the kernel has TW = 4 or 8 waves: with
// 8, waves 4-7 only join the tile's barriers and add their threads to the publish, phase B's
// loads and phase C (PRL_UPD_SPL_WAVES; A/B)
constexpr int SPL_NW = 4;
constexpr int SPL_CQ = 4;   // quads per norm piece (spl_piece)

// The trunk's forward of channel block b (H0^T = W0 X^T, GroupNorm + SiLU) for one tile's
// inputs: F block b into the LDS tile Fs, the normalised values and 1 / std kept for the backward.
template <int KSM>
__device__ __forceinline__ void spl_trunk_fwd(const UpdNet& n, const float* W, const UpdScr& sc,
                                              const float (&xin)[KSM], upd_v4& xh0, float& r0) {
  const int l = threadIdx.x & 63, x = l & 15, q = l >> 4, b = threadIdx.x >> 6;
  const int D = n.D, KS = (D + 3) >> 2;
  upd_v4 acc = {0.f, 0.f, 0.f, 0.f}, Fw;
  const float* wr = W + n.w0.lds + (16 * b + x) * n.w0.stride;
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
    if (s < KS) {
      const int d = 4 * s + q;
      acc = upd_mma(d < D ? wr[d] : 0.0f, xin[s], acc);
    }
  }
  upd_gn_fwd_frag(acc, upd_ld4(W + n.g0.lds + 16 * b + 4 * q), upd_ld4(W + n.b0.lds + 16 * b + 4 * q), xh0, r0,
                  Fw);
  upd_st4(sc.Fs + x * UPD_ZS + 16 * b + 4 * q, Fw);
}

// one 16-row tile of role r = head h (h = r): forward (trunk + head h), the head's loss, its
// backward through the trunk; the gradient into the LDS image Ga (first tile of the step: every
// entry the role publishes is stored, never accumulated, since a split workgroup runs ONE tile
// per step).  Three workgroup barriers.  PRE: the trunk's forward ran already (spl_trunk_fwd at
// the end of the previous step's AdamW, WB form): its Fs block is in LDS, xh0 / r0 are given.
template <int KA, int TW, bool PRE = false>
__device__ __forceinline__ void spl_tile(const UpdNet& n, const UpdArgs& args, int h, const float* W,
                                         float* Ga, const UpdScr& sc, const UpdIn<upd_ksm<KA>()>& in,
                                         int rc, float invB, unsigned long long* tm, bool direct,
                                         __amdgpu_buffer_rsrc_t rs_mypart, upd_v4 pxh0 = upd_v4{},
                                         float pr0 = 0.f) {
  constexpr int KSM = upd_ksm<KA>();
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  if (TW > SPL_NW && w >= SPL_NW) {   // the tile's three barriers, nothing else
    __syncthreads();
    __syncthreads();
    __syncthreads();
    return;
  }
  const int b = w;
  const int D = n.D, KS = (D + 3) >> 2;
  const bool timer = args.profile && blockIdx.x == 0 && t == 0;
  unsigned long long tl = timer ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // (profile: from the previous phase mark to the tile's start — the loop top and the prefetch)
  if (timer) tm[11] += tl - tm[31];   // tm[31] = pts[7] (hdr + 64), the last phase mark
#define SPL_CMARK(i)                                                   \
  if (timer) {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
    tm[i] += now_ - tl;                                                \
    tl = now_;                                                         \
  }
  const UpdHead hi = upd_head_info(n, h);
  const int oc = hi.oc, no = hi.no;
  // ---- forward: trunk block b (H0^T = W0 X^T, GroupNorm + SiLU), every wave its own block
  upd_v4 xh0, xh, G;
  float r0, rh;
  if constexpr (PRE) {
    xh0 = pxh0;
    r0 = pr0;
  } else {
    spl_trunk_fwd<KSM>(n, W, sc, in.xin, xh0, r0);
  }
  __syncthreads();   // #0: Fs
  {
    upd_v4 F[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) F[bb] = upd_ld4(sc.Fs + x * UPD_ZS + 16 * bb + 4 * q);
    // head h block b: Z^T = W1_h[16b ..][:] F^T — ONE accumulation chain in the order of
    // upd_tile_fwd (the evaluate kernel's), so the first minibatch's ratio is exactly 1
    upd_v4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const upd_v4 wa = upd_ld4(W + hi.w1 + (16 * b + x) * UPD_HS + 16 * bb + 4 * q);
      z = upd_mma(wa[0], F[bb][0], z);
      z = upd_mma(wa[1], F[bb][1], z);
      z = upd_mma(wa[2], F[bb][2], z);
      z = upd_mma(wa[3], F[bb][3], z);
    }
    upd_gn_fwd_frag(z, upd_ld4(W + hi.g1 + 16 * b + 4 * q), upd_ld4(W + hi.b1 + 16 * b + 4 * q), xh, rh, G);
    // output layer partial over this block's 16 channels: O^T[j][row] += W2[j][16b + 4q + i] G^T
    const bool mine = x >= oc && x < oc + no;
    const upd_v4 wv = mine ? upd_ld4(W + hi.w2 + (x - oc) * UPD_HS + 16 * b + 4 * q) : upd_v4{0.f, 0.f, 0.f, 0.f};
    upd_v4 o = {0.f, 0.f, 0.f, 0.f};
    o = upd_mma(wv[0], G[0], o);
    o = upd_mma(wv[1], G[1], o);
    o = upd_mma(wv[2], G[2], o);
    o = upd_mma(wv[3], G[3], o);
    upd_st4(sc.Op + (w * 16 + x) * 16 + 4 * q, o);   // [w][row x][j = 4q + i]
    if (t < UPD_RT * UPD_RIN) sc.Rin[t] = in.rin;
  }
  SPL_CMARK(0)
  __syncthreads();   // #1: Op, Rin
  SPL_CMARK(1)
  // ---- the head's per-row loss on lanes q == 0 of every wave (each wave needs dO; one wave per
  //      SIMD, so the redundant chains do not share issue slots): the actor's surrogate chain
  //      (dO of the actor's outputs, lp[0] = -min(s1, s2), lp[2] = H) or the critic's SmoothL1
  //      (dO of V, lp[1]) — the same arithmetic as the other forms (upd_row_loss)
  float lp[3] = {0.f, 0.f, 0.f};
  float* dOrow = sc.dOs + (w * 16 + x) * 16;
  {
    float O[UPD_MAXO], dO[UPD_MAXO];
    upd_tile_outputs_reg<SPL_NW>(n, W, sc, O);
    if (q == 0) {
      if (x < rc) {
        if (h == 0)
          upd_row_loss<1, KA, 2>(n, O, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dO, lp);
        else
          upd_row_loss<1, KA, 1>(n, O, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dO, lp);
      } else {
#pragma unroll
        for (int j = 0; j < UPD_MAXO; ++j) dO[j] = 0.f;
      }
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        if (4 * j4 < n.nout) upd_st4(dOrow + 4 * j4, upd_v4{dO[4 * j4], dO[4 * j4 + 1], dO[4 * j4 + 2], dO[4 * j4 + 3]});
    }
  }
  const float* dOw = sc.dOs + w * 16 * 16;
  float* Tw = sc.Ts + w * upd_ts(n) * UPD_RT * 16;
  upd_st4(Tw + x * 16 + 4 * q, G);   // G transposed for dW2 (rows x channels of block b)
  upd_wave_sync();
  SPL_CMARK(2)
  {
    // dW2_h[j][16b + x] = sum_rows dO[row][oc + j] G[row][16b + x]; dG^T block b = W2_h^T dO_h^T
    // (K = the head's outputs) — every operand (and γ1 / β1) read first, in flight together
    float oa[4], tb[4], ga[UPD_MAXA / 4], gb[UPD_MAXA / 4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      oa[s] = x < no ? dOw[(4 * s + q) * 16 + oc + x] : 0.0f;
      tb[s] = Tw[(4 * s + q) * 16 + x];
    }
#pragma unroll
    for (int s = 0; s < UPD_MAXA / 4; ++s) {
      const int j = 4 * s + q;
      ga[s] = j < no ? W[hi.w2 + j * UPD_HS + 16 * b + x] : 0.0f;
      gb[s] = j < no ? dOw[x * 16 + oc + j] : 0.0f;
    }
    const upd_v4 g1w = upd_ld4(W + hi.g1 + 16 * b + 4 * q), b1w = upd_ld4(W + hi.b1 + 16 * b + 4 * q);
    __builtin_amdgcn_sched_barrier(0);
    upd_v4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = upd_mma(oa[s], tb[s], acc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * q + i < no) Ga[hi.w2 + (4 * q + i) * UPD_HS + 16 * b + x] = acc[i];
    // GroupNorm + SiLU backward -> dZ
    upd_v4 dg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < UPD_MAXA / 4; ++s)
      if (4 * s < no) dg = upd_mma(ga[s], gb[s], dg);
    upd_v4 dy;
    const upd_v4 dz = upd_gn_bwd_frag(dg, xh, g1w, b1w, rh, dy);
    upd_st4(sc.Zs + x * UPD_ZS + 16 * b + 4 * q, dz);
    upd_v4 dyx;
#pragma unroll
    for (int i = 0; i < 4; ++i) dyx[i] = dy[i] * xh[i];
    upd_colsum_add(dyx, Ga + hi.g1 + 16 * b + 4 * q, x == 0, true);
    upd_colsum_add(dy, Ga + hi.b1 + 16 * b + 4 * q, x == 0, true);
  }
  // inputs, rows x features, for dW0
#pragma unroll
  for (int s = 0; s < KSM; ++s)
    if (s < KS && (s % SPL_NW) == w) sc.Xs[x * sc.XS + 4 * s + q] = in.xin[s];
  SPL_CMARK(3)
  __syncthreads();   // #2: Zs, Xs
  SPL_CMARK(4)
  {
    // ---- dF^T block b = W1_h^T dZ^T first (it heads the trunk's chain: GroupNorm backward ->
    //      dW0), K = 64 head channels permuted so the A reads are conflict-free
    const float* Zh = sc.Zs + x * UPD_ZS;
    const float* Wh = W + hi.w1 + 16 * b + x;
    upd_v4 zb[4];
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) zb[sg] = upd_ld4(Zh + 16 * sg + 4 * q);
    upd_v4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
    float wa[16];   // (the A operands read first, in flight together with zb: see dW1 below)
#pragma unroll
    for (int s = 0; s < 16; ++s) wa[s] = Wh[(16 * (s & 3) + 4 * q + (s >> 2)) * UPD_HS];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) d1 = upd_mma(wa[s], zb[s & 3][s >> 2], d1);
      else d0 = upd_mma(wa[s], zb[s & 3][s >> 2], d0);
    }
    // ---- dW1_h[16b + 4q + i][16bb + x] = sum_rows dZ[row][16b + 4q + i] F[row][16bb + x]:
    //      independent of dF, issued behind it
    upd_v4 acc[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) acc[bb] = upd_v4{0.f, 0.f, 0.f, 0.f};
    // every operand read first, in flight together (the scheduler otherwise issued them two by two
    // between the MFMAs, one LDS round trip per pair under the kernel's register pressure)
    float za[4], fb[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      za[s] = sc.Zs[(4 * s + q) * UPD_ZS + 16 * b + x];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) fb[s][bb] = sc.Fs[(4 * s + q) * UPD_ZS + 16 * bb + x];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) acc[bb] = upd_mma(za[s], fb[s][bb], acc[bb]);
    }
    upd_v4 dF;
#pragma unroll
    for (int i = 0; i < 4; ++i) dF[i] = d0[i] + d1[i];
    // trunk GroupNorm + SiLU backward of THIS head's share -> dH0 (block b), γ0 / β0 sums
    upd_v4 dy0;
    const upd_v4 dH0 = upd_gn_bwd_frag(dF, xh0, upd_ld4(W + n.g0.lds + 16 * b + 4 * q),
                                       upd_ld4(W + n.b0.lds + 16 * b + 4 * q), r0, dy0);
    upd_v4 dyx;
#pragma unroll
    for (int i = 0; i < 4; ++i) dyx[i] = dy0[i] * xh0[i];
    upd_colsum_add(dyx, Ga + n.g0.lds + 16 * b + 4 * q, x == 0, true);
    upd_colsum_add(dy0, Ga + n.b0.lds + 16 * b + 4 * q, x == 0, true);
    if (direct) {
      // dW1 (16 of the role's ~20 KB) straight from the accumulators into this tile group's
      // partial (4-B sc1 stores, 64-B runs per 16 lanes), under the trunk backward below, instead
      // of through the LDS image and the publish loop (PRL_UPD_SPL_DIRECT, A/B)
      const int k0 = hi.w1 + (16 * b + 4 * q) * UPD_HS + x;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int i = 0; i < 4; ++i) st1_sc1(rs_mypart, k0 + i * UPD_HS + 16 * bb, acc[bb][i]);
    } else {
      float* gw1 = Ga + hi.w1 + (16 * b + 4 * q) * UPD_HS + x;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int i = 0; i < 4; ++i) gw1[i * UPD_HS + 16 * bb] = acc[bb][i];
    }
    SPL_CMARK(5)
    // ---- dW0[16b + 4q + i][16e + x] = sum_rows dH0[row][ch] X[row][d] (dH0 transposed via Tw;
    //      Tw's G was last read by this wave's dW2 before barrier #2)
    upd_st4(Tw + x * 16 + 4 * q, dH0);
    upd_wave_sync();
#pragma unroll
    for (int e = 0; e < (KSM + 3) / 4; ++e) {
      if (16 * e < D) {
        upd_v4 a0 = {0.f, 0.f, 0.f, 0.f};
        const int d = 16 * e + x;
        float ta[4], xb[4];   // (operands read first, in flight together)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          ta[s] = Tw[(4 * s + q) * 16 + x];
          xb[s] = d < D ? sc.Xs[(4 * s + q) * sc.XS + d] : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) a0 = upd_mma(ta[s], xb[s], a0);
        if (d < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i) Ga[n.w0.lds + (16 * b + 4 * q + i) * n.w0.stride + d] = a0[i];
        }
      }
    }
  }
  SPL_CMARK(6)
  // ---- the head's output biases and loss partials, spread over waves 1-3 (every wave holds the
  //      same dO rows and lp lanes; the tile's last barrier waits for the slowest wave): wave 1
  //      the biases, wave 2 loss partial k = 0 or 1 (the actor's surrogate / the critic's
  //      SmoothL1), wave 3 the actor's entropy partial k = 2
  if (w == 1 && l < no) {   // f64 sum: the softmax outputs' dO cancel across rows
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < UPD_RT; ++r) acc += (double)dOw[r * 16 + oc + l];
    Ga[(h == 0 ? n.b2[0].lds : n.b2[1].lds) + l] = (float)acc;
  }
  if (w == 2) {
    const int k = h == 0 ? 0 : 1;
    const float s = upd_rsum16(lp[k]);
    if (l == 0) Ga[n.Lp + k] = s;
  }
  if (w == 3 && h == 0) {
    const float s = upd_rsum16(lp[2]);
    if (l == 0) Ga[n.Lp + 2] = s;
  }
  SPL_CMARK(7)
#undef SPL_CMARK
}

// Phase B's slices, balanced by loads: a trunk or loss quad sums 2 Gt partials, a head quad Gt,
// and phase B's time per workgroup follows the bytes it loads (~20 KB per us per CU, measured:
// equal-quad slices left the trunk's owners loading twice the others' bytes, 3.7 vs 2.0 us).
// So a head quad weighs 4 units and a trunk / loss quad tw4 (8 = twice: the default;
// PRL_UPD_SPL_TW4 for A/Bs): weighted position w(q) = 4 q + (tw4 - 4) min(q, QT), U = 4 (Qp - QT)
// + tw4 (QT + 1) units, and slice g starts at the first quad with w(q) >= U g / G, rounded down
// to a multiple of SPL_CQ (a norm piece's chunk, below: no chunk straddles two slices).  The
// host's slice-owner check (upd_split_own) cuts the same way.
__host__ __device__ inline int spl_slice_start(int g, int G, int Qp, int QT, int tw4 = 8) {
  const int Qtot = Qp + 1;
  const int64_t U = 4 * (int64_t)(Qp - QT) + (int64_t)tw4 * (QT + 1);
  const int64_t u = U * g / G, ut = (int64_t)tw4 * QT;
  const int64_t q = u <= ut ? (u + tw4 - 1) / tw4 : QT + (u - ut + 3) / 4;
  return q < Qtot ? (int)(q / SPL_CQ) * SPL_CQ : Qtot;
}

// Norm pieces (PRL_UPD_SPL_PIECES, default on): clip_grad_norm_'s squared norm as a sum of
// per-chunk pieces, chunk c = reduced-gradient quads [SPL_CQ c, SPL_CQ c + SPL_CQ) below the loss
// quad, piece = ((q0^2 + q1^2) + (q2^2 + q3^2)) of the quads' ((x^2 + y^2) + (z^2 + w^2)).  Each
// piece is a function of its chunk's reduced values only, formed by whichever workgroup owns the
// chunk (slice owner, helper, or the data-parallel union of the slice), so every launch form
// gives the same pieces; phase C sums them in one canonical order (the same bits on every
// workgroup) and loads only the gradient quads its role owns (trunk + its head: ~half the
// gradient) instead of all of them.
// (upd_sq4 / upd_piece, prl_ppo_update.hip: shared with the data-parallel union slices; SPL_CQ = 4)

// Sum of quad q over partials first, first + stride, ... of part (< Gt) and, for a dual quad
// (nv = 2 Gt: the trunk / loss quads), over the same positions of part2 (quad qd there): the
// part and part2 loads of a chunk are issued together (one memory round trip), each from its own
// WAVE-UNIFORM buffer resource (a per-lane choice of resource compiles to a waterfall loop per
// load), with 32-bit byte offsets stepped by a uniform stride.  Order: chunk by chunk, part's
// partials then part2's (deterministic).
__device__ inline void spl_sum_partials(__amdgpu_buffer_rsrc_t rs_part, __amdgpu_buffer_rsrc_t rs_part2,
                                        int Qtot, int P2, int q, int qd, int first, int stride,
                                        int Gt, int nv, double& ax, double& ay, double& az,
                                        double& aw) {
  constexpr int NB = 8;
  const bool dual = nv > Gt;
  const unsigned d1 = (unsigned)stride * (unsigned)Qtot * 16u, d2 = (unsigned)stride * (unsigned)P2 * 16u;
  for (int v0 = first; v0 < Gt; v0 += NB * stride) {
    const unsigned o1 = ((unsigned)v0 * (unsigned)Qtot + (unsigned)q) * 16u;
    const unsigned o2 = ((unsigned)v0 * (unsigned)P2 + (unsigned)qd) * 16u;
    v4u a[NB], b[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (v0 + u * stride < Gt) a[u] = __builtin_amdgcn_raw_buffer_load_b128(rs_part, o1 + (unsigned)u * d1, 0, UPD_AUX_SC1);
    if (dual) {
#pragma unroll
      for (int u = 0; u < NB; ++u)
        if (v0 + u * stride < Gt) b[u] = __builtin_amdgcn_raw_buffer_load_b128(rs_part2, o2 + (unsigned)u * d2, 0, UPD_AUX_SC1);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (v0 + u * stride < Gt) {
        ax += __uint_as_float(a[u].x); ay += __uint_as_float(a[u].y);
        az += __uint_as_float(a[u].z); aw += __uint_as_float(a[u].w);
      }
    }
    if (dual) {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (v0 + u * stride < Gt) {
          ax += __uint_as_float(b[u].x); ay += __uint_as_float(b[u].y);
          az += __uint_as_float(b[u].z); aw += __uint_as_float(b[u].w);
        }
      }
    }
  }
}

// Profile only (PRL_UPD_PROFILE=1, every 16th step: A at s = 0 mod 16, B at 8 mod 16): arrival
// skew at counter `slot` (0: A, 1: B).
// Each workgroup stamps its arrival (prof[32 + 256 slot + g]); after the wait, workgroup 0's
// wave 0 reads the stamps back (one extra round trip on the sampled steps, kept out of the
// phase marks) and sums the last arrival - its own and the last - the first into
// tm[12 + 2 slot], tm[13 + 2 slot]; tm[16] counts the samples, tm[17] those whose last arrival
// at A was a role-1 (critic) workgroup.
__device__ inline void spl_prof_stamp(const UpdArgs& a, int slot, int g) {
  __hip_atomic_store(upd_g(a.prof + 32 + 256 * slot + g), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void spl_prof_skew(const UpdArgs& a, int slot, int G, int Gt, unsigned long long* tm) {
  const int l = threadIdx.x & 63;
  unsigned long long mx = 0ull, mn = ~0ull, own = 0ull;
  int arg = 0;
  for (int i0 = 0; i0 < G && i0 < 256; i0 += 64) {
    const int i = i0 + l;
    const unsigned long long v = i < G ? __hip_atomic_load(upd_g(a.prof + 32 + 256 * slot + i), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    unsigned long long vmx = i < G ? v : 0ull, vmn = i < G ? v : ~0ull;
    int vi = i;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long ox = __shfl_xor(vmx, o), on = __shfl_xor(vmn, o);
      const int oi = __shfl_xor(vi, o);
      if (ox > vmx || (ox == vmx && oi < vi)) { vmx = ox; vi = oi; }
      vmn = on < vmn ? on : vmn;
    }
    if (i0 == 0) own = __shfl(v, 0);
    if (vmx > mx) { mx = vmx; arg = vi; }
    mn = vmn < mn ? vmn : mn;
  }
  if (l == 0 && mx >= own && mx >= mn) {
    tm[12 + 2 * slot] += mx - own;
    tm[13 + 2 * slot] += mx - mn;
    if (slot == 0) {
      tm[16] += 1ull;
      tm[17] += arg >= Gt ? 1ull : 0ull;
    }
  }
}

// The slice and this thread's place in it are loop-invariant: planned once before the step
// loop (64-bit and integer divisions: ~0.1 us of dependent instructions per step otherwise).
struct SplSlice {
  int qlo, qhi, nq;
  int spl;      // threads per quad (narrow slices)
  int qi, sb;   // this thread's quad (qlo + qi) and its first partial
};
template <int NT>
__device__ inline SplSlice spl_slice_plan(int g, int G, int Qp, int QT, int Gt, int fill, int tw4 = 8) {
  SplSlice p;
  p.qlo = spl_slice_start(g, G, Qp, QT, tw4);
  p.qhi = spl_slice_start(g + 1, G, Qp, QT, tw4);
  p.nq = p.qhi - p.qlo;
  // spl threads per quad, each summing every spl-th partial: a power of two (fill 0), or as
  // many as the NT threads allow (fill 1: more loads in flight; the slice loads are latency-bound)
  int spl = 1;
  if (p.nq > 0) {
    if (fill) spl = std::max(1, std::min(Gt, NT / p.nq));
    else
      while (spl * 2 * p.nq <= NT && spl * 2 <= Gt) spl *= 2;
  }
  p.spl = spl;
  const int t = threadIdx.x;
  p.qi = p.nq > 0 ? t % p.nq : 0;
  p.sb = p.nq > 0 ? t / p.nq : 0;
  return p;
}
// Phase B of the split form: slice g of G (spl_slice_start) over the Gt role partials; the
// trunk quads [0, QT) and the loss quad Qp also over part2 (role 1's trunk partials,
// [Gt][QT + 1] quads).  Per quad: part[0 .. Gt) then part2[0 .. Gt) in the order sub,
// sub + spl, ... for each of spl threads, combined in sub order (deterministic).
template <int NT>
__device__ inline void spl_slice_reduce(__amdgpu_buffer_rsrc_t rs_part, __amdgpu_buffer_rsrc_t rs_part2,
                                        __amdgpu_buffer_rsrc_t rs_red, int Qtot, int Qp, int QT,
                                        const SplSlice& pl, int Gt, float* scratch, bool sys,
                                        UpdSub sub, const UpdArgs& args, int par,
                                        float4* gout = nullptr, float* pieces = nullptr) {
  // gout (the slice-owner form, narrow slices only): thread t < nq keeps its quad's reduced
  // gradient in *gout instead of storing it (the loss quad Qp is stored as always); pieces: the
  // norm pieces of the slice's chunks (not with sys: the data-parallel union forms them)
  const int t = threadIdx.x;
  const int qlo = pl.qlo, qhi = pl.qhi, nq = pl.nq;
  if (nq <= 0) return;
  const int P2 = QT + 1;
  auto fin = [&](int q, const float4 r) {
    if (sys && args.dp_push) {
      // push form: straight into every rank's receive slot [par][this rank] (upd_dp_union_slice_push)
#pragma unroll
      for (int rr = 0; rr < UPD_MAX_RANKS; ++rr)
        if (rr < args.world)
          st4_aux<UPD_AUX_SYS>(upd_rsrc(args.xbuf[rr] + args.xpush_off +
                                        ((size_t)par * UPD_MAX_RANKS + args.rank) * Qtot * 4),
                               (size_t)q * 4, r);
    } else if (sys) {
      st4_aux<UPD_AUX_SYS>(rs_red, (size_t)q * 4, r);   // data-parallel: the rank's slice buffer
    } else {
      st4_sc1(rs_red, (size_t)q * 4, r);
    }
  };
  if (2 * nq > NT) {
    // wide slices (few workgroups, small minibatches): each thread owns whole quads (uniform
    // trip count: the pieces' DPP sums need every lane)
    for (int q0 = qlo; q0 < qhi; q0 += NT) {
      const int q = q0 + t;
      float sqv = 0.f;
      if (q < qhi) {
        double ax = 0.0, ay = 0.0, az = 0.0, aw = 0.0;
        const bool dual = q < QT || q == Qp;
        spl_sum_partials(rs_part, rs_part2, Qtot, P2, q, q < QT ? q : QT, 0, 1, Gt, dual ? 2 * Gt : Gt,
                         ax, ay, az, aw);
        const float4 r = float4{(float)ax, (float)ay, (float)az, (float)aw};
        fin(q, r);
        sqv = q < Qp ? upd_sq4(r) : 0.f;
      }
      if (pieces) upd_piece(pieces, sqv, q, q < qhi && q < Qp);
    }
    return;
  }
  const int spl = pl.spl;
  double* red = reinterpret_cast<double*>(scratch);   // [spl][nq][4]
  if (t < spl * nq) {
    const int qi = pl.qi, sb = pl.sb, q = qlo + qi;
    double ax = 0.0, ay = 0.0, az = 0.0, aw = 0.0;
    const bool dual = q < QT || q == Qp;
    spl_sum_partials(rs_part, rs_part2, Qtot, P2, q, q < QT ? q : QT, sb, spl, Gt, dual ? 2 * Gt : Gt,
                     ax, ay, az, aw);
    double* o = red + 4 * (sb * nq + qi);
    o[0] = ax; o[1] = ay; o[2] = az; o[3] = aw;
  }
  sub.mark(0);   // thread 0's partial loads landed and summed
  __syncthreads();
  float sqv = 0.f;
  if (t < nq) {
    double ax = red[4 * t], ay = red[4 * t + 1], az = red[4 * t + 2], aw = red[4 * t + 3];
    for (int k = 1; k < spl; ++k) {
      const double* o = red + 4 * (k * nq + t);
      ax += o[0]; ay += o[1]; az += o[2]; aw += o[3];
    }
    const float4 r = float4{(float)ax, (float)ay, (float)az, (float)aw};
    if (gout && qlo + t != Qp) *gout = r;
    else fin(qlo + t, r);
    sqv = qlo + t < Qp ? upd_sq4(r) : 0.f;
  }
  if (pieces) upd_piece(pieces, sqv, qlo + t, t < nq && qlo + t < Qp);
  sub.mark(1);   // slice combined, its stores issued
}

// The split form's counter waits (PRL_UPD_SPL_POLL, A/B): 0 = one poll in flight, s_sleep 1
// between polls (default); 1 = four polls in flight; 2 / 3 / 4 = one in flight, s_sleep 2 / 4 / 8
// (fewer polls against the counter lines while the other workgroups' arrivals land there)
__device__ inline bool spl_wait(const UpdArgs& args, int base, unsigned target) {
  switch (args.spl_poll) {
    case 1: return upd_wait_sharded_pipe(args.ctr, base, target);
    case 2: return upd_wait_sharded<2>(args.ctr, base, target);
    case 3: return upd_wait_sharded<4>(args.ctr, base, target);
    case 4: return upd_wait_sharded<8>(args.ctr, base, target);
    default: return upd_wait_sharded<1>(args.ctr, base, target);
  }
}

// Phase-B helpers: workgroups G .. Gs - 1 of a single-GPU split launch (PRL_UPD_SPL_HELP; by
// default the CUs the 2 Gt tile workgroups leave idle).  They hold no parameters and run no tile:
// each step they wait for counter A, reduce their slice, and arrive at counter B.  The slices are
// cut over all Gs owners (spl_slice_start), so an owner loads ~1 / Gs of the partials' bytes
// instead of ~1 / G: phase B's landing is the per-CU rate of latency-bound sc1 loads (~20 KB per
// us), not the chip's.  Each quad is still summed over the same partials in the same order, and
// the reduced gradient lands in the same place, so the tile workgroups see the same hand-off.
template <int NT>
__device__ __forceinline__ void spl_helper(const UpdArgs& args, int g, int Qtot, int Qp, int QT, float* scratch,
                                        int* s_abort) {
  const int t = threadIdx.x;
  const SplSlice slc = spl_slice_plan<NT>(g, args.Gs, Qp, QT, args.Gt, args.spl_fill, args.spl_tw4);
  const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_part2 = upd_rsrc(args.part2),
                               rs_red = upd_rsrc(args.red);
  const UpdSub none{nullptr, nullptr};
  for (int s = 0; s < args.total_steps; ++s) {
    if (t < 64) {
      const bool ok = upd_wait_sharded(args.ctr, UPD_CTR_A, (unsigned)args.G * (unsigned)(s + 1));
      if (t == 0) *s_abort = ok ? 0 : 1;
    }
    __syncthreads();
    if (*s_abort) return;
    spl_slice_reduce<NT>(rs_part, rs_part2, rs_red, Qtot, Qp, QT, slc, args.Gt, scratch, false, none, args, 0,
                         nullptr, args.spl_pieces ? args.sq : nullptr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      if (args.profile && (s & 15) == 8) spl_prof_stamp(args, 1, g);
      upd_arrive(args.ctr, UPD_CTR_B, g);
    }
  }
}

// Wave-block AdamW (WB: the 4-wave workgroup-AdamW form).  Before barrier #0 a tile's wave b
// reads only the parameters of its own channel block — W0 rows 16b .. 16b + 15, γ0 / β0 block b,
// the head's W1 rows 16b .. 16b + 15, γ1 / β1 block b, W2 columns 16b .. 16b + 15 — and every
// other parameter read comes after barrier #0.  So when wave b's AdamW updates exactly those
// quads (wave 1 also the head's output biases, read after barrier #1), no workgroup barrier is
// needed between AdamW and the next step's tile: a wave goes from its last AdamW slot straight
// into its forward.  The same lists are what each wave WRITES into the tile's gradient image
// (spl_tile: dW2 / γ1 β1 / dW1 / γ0 β0 / dW0 of its block; wave 1 the output biases), so each
// wave also publishes its own list straight after its tile, without a workgroup barrier in front
// (the loss partials' words go out from the waves that form them: 2 and 3).  List k of (role h, wave b) -> parameter quad (-1 past its end); lane l
// holds entries l + 64 i (SPL_WBQ slots; the host checks the length).  W1 / W2 padding columns
// (zero gradient, zero moments: they stay 0) are not listed.
constexpr int SPL_WBQ = 5;
__host__ __device__ constexpr int spl_wb_len(const UpdNet& n, int h, int b) {
  return 4 * n.w0.stride + 8 + 16 * UPD_H / 4 + 8 + 4 * n.out[h] + (b == 1 ? (n.out[h] + 3) / 4 : 0);
}
__host__ __device__ __forceinline__ int spl_wb_quad(const UpdNet& n, int h, int b, int k) {
  const int s0 = 4 * n.w0.stride;   // W0 rows 16b .. 16b + 15: 16 stride floats, contiguous
  if (k < s0) return (n.w0.lds + 16 * b * n.w0.stride) / 4 + k;
  k -= s0;
  if (k < 4) return (n.g0.lds + 16 * b) / 4 + k;
  k -= 4;
  if (k < 4) return (n.b0.lds + 16 * b) / 4 + k;
  k -= 4;
  const int w1 = h == 0 ? n.w1[0].lds : n.w1[1].lds;   // (two-head nets: h is 0 or 1)
  if (k < 256) return (w1 + (16 * b + (k >> 4)) * UPD_HS) / 4 + (k & 15);
  k -= 256;
  if (k < 4) return ((h == 0 ? n.g1[0].lds : n.g1[1].lds) + 16 * b) / 4 + k;
  k -= 4;
  if (k < 4) return ((h == 0 ? n.b1[0].lds : n.b1[1].lds) + 16 * b) / 4 + k;
  k -= 4;
  const int no = h == 0 ? n.out[0] : n.out[1];
  if (k < 4 * no) return ((h == 0 ? n.w2[0].lds : n.w2[1].lds) + (k >> 2) * UPD_HS + 16 * b) / 4 + (k & 3);
  k -= 4 * no;
  if (b == 1 && k < (no + 3) / 4) return (h == 0 ? n.b2[0].lds : n.b2[1].lds) / 4 + k;
  return -1;
}
// Host check (once per net shape, prl_ppo_update): role h's four lists cover every quad the
// role owns (trunk + head h) exactly once, W1 / W2 padding quads aside, within SPL_WBQ slots.
inline bool spl_wb_check(const UpdNet& n) {
  if (n.nh != 2) return false;
  const int Qp = n.Lp / 4, QT = n.w1[0].lds / 4, QH = n.w1[1].lds / 4;
  for (int h = 0; h < 2; ++h) {
    std::vector<int> seen(Qp, 0);
    for (int b = 0; b < 4; ++b) {
      if (spl_wb_len(n, h, b) > 64 * SPL_WBQ) return false;
      for (int k = 0; k < 64 * SPL_WBQ; ++k) {
        const int q = spl_wb_quad(n, h, b, k);
        if ((q >= 0) != (k < spl_wb_len(n, h, b))) return false;
        if (q < 0) continue;
        if (q >= Qp || seen[q]++) return false;
      }
    }
    for (int q = 0; q < Qp; ++q) {
      const bool owned = h == 0 ? q < QH : (q < QT || q >= QH);
      // a padding quad: columns 64 .. 67 of a W1 / W2 row (stride UPD_HS = 68)
      bool pad = false;
      for (int hh = 0; hh < 2; ++hh) {
        const int lo = (4 * q - n.w1[hh].lds), lo2 = (4 * q - n.w2[hh].lds);
        if (lo >= 0 && lo < UPD_H * UPD_HS && lo % UPD_HS == UPD_H) pad = true;
        if (lo2 >= 0 && lo2 < n.out[hh] * UPD_HS && lo2 % UPD_HS == UPD_H) pad = true;
      }
      if (seen[q] != ((owned && !pad) ? 1 : 0)) return false;
    }
  }
  return true;
}

// NQC = ceil(Qp / 256): quads per thread of phase C's canonical sweep (the moment registers
// cover the same slots; a slot holds moments only where this role owns the quad).
// DP: data-parallel ranks (prl_ppo_update_dpx): union-minibatch row weights inv_count[j] and,
// after phase B, the cross-rank sum of each slice (upd_dp_union_slice, as the 8-wave kernel);
// the 2 Gt workgroups of every rank cut the gradient into the same 2 Gt slices.
// OWN: the slice-owner form (one rank, narrow slices: every workgroup's slice has at most NT / 2
// quads).  The owner of a slice quad keeps that quad's AdamW moments and runs its AdamW in phase
// B, with clip coefficient 1, and publishes the NEW WEIGHTS (and its waves' pieces of the clip
// norm) instead of the gradient; phase C loads the weights into LDS.  So AdamW runs once per quad
// on the chip (one quad per owning thread) instead of once per workgroup over ~1,185 quads, and
// no workgroup holds moment registers for the whole net.  clip_grad_norm_ scales a step only when
// the norm (summed from the pieces in one fixed order, the same on every workgroup) exceeds
// max_norm: then every workgroup sees it, the owners redo their quads from the kept gradient,
// moments and the LDS weights (not yet replaced) with the true coefficient, and one more
// hand-off (counter C, the corrected weights in red_c) follows.  The same AdamW arithmetic per
// element as the workgroup form, so the same bits whenever the clip coefficient is the same.
template <int NQC, int KA, bool DP, int TW, bool OWN = false>
__device__ __forceinline__ void ppo_split_body(const UpdNet& n, const UpdArgs& args) {
  constexpr int SPL_NT = 64 * TW;
  extern __shared__ __align__(16) float upd_lds[];
  const int t = threadIdx.x, g = blockIdx.x, G = args.G, Gt = args.Gt;
  const int role = g / Gt, gt = g - role * Gt;   // role = the head this workgroup runs
  const int Lp = n.Lp, Qp = Lp / 4, Qtot = Qp + 1;
  const int QT = n.w1[0].lds / 4;   // trunk quads [0, QT)
  const int QH = n.w1[1].lds / 4;   // head 0: [QT, QH), head 1: [QH, Qp)
  // owned quads: the trunk and this role's head (the only parameters its tile reads)
  auto owned = [&](int q) { return role == 0 ? q < QH : (q < QT || q >= QH); };
  // slot i of this thread: the quad of the canonical sweep (t + NT i) its moments / AdamW cover,
  // where this role owns it (-1: none)
  // WB: the wave-block lists (spl_wb_quad) instead of the canonical sweep
  constexpr bool WB = TW == SPL_NW && !OWN;
  int wq[SPL_WBQ];
  if constexpr (WB) {
#pragma unroll
    for (int i = 0; i < SPL_WBQ; ++i) wq[i] = spl_wb_quad(n, role, t >> 6, (t & 63) + 64 * i);
  }
  auto slotq = [&](int i) {
    if constexpr (WB) return wq[i];
    const int o = t + i * SPL_NT;
    return (o < Qp && owned(o)) ? o : -1;
  };
  float* hdr = upd_lds;
  float* scratch = upd_lds + UPD_HDR;
  const int scr_floats = (upd_scratch_floats(n.D, SPL_NW, upd_ts(n)) + 3) & ~3;
  float* W = scratch + scr_floats;   // [Lp]
  float* Ga = W + Lp;                // [Lp + 4]
  const UpdScr sc = upd_scr(scratch, n.D, SPL_NW);
  int* s_abort = reinterpret_cast<int*>(hdr + 8);
  float* s_adam = hdr + 10;
  const int Gs = args.Gs;   // slice owners: the G tile workgroups, then Gs - G phase-B helpers
  if (g >= G) {
    spl_helper<SPL_NT>(args, g, Qtot, Qp, QT, scratch, s_abort);
    return;
  }

  constexpr int NMR = OWN ? 1 : (WB ? SPL_WBQ : NQC);   // moment slots per thread
  float4 mreg[NMR], vreg[NMR];
  for (int q = t; q < Qp; q += SPL_NT)
    *reinterpret_cast<float4*>(W + 4 * q) = *reinterpret_cast<const float4*>(args.params + 4 * q);
  // OWN: this thread's slice quad (see slc below) and its moments
  const SplSlice slc0 = spl_slice_plan<SPL_NT>(g, Gs, Qp, QT, Gt, args.spl_fill, args.spl_tw4);
  const int oq = (OWN && t < slc0.nq && slc0.qlo + t < Qp) ? slc0.qlo + t : -1;
  if constexpr (OWN) {
    mreg[0] = oq >= 0 ? *reinterpret_cast<const float4*>(args.exp_avg + 4 * oq) : float4{0.f, 0.f, 0.f, 0.f};
    vreg[0] = oq >= 0 ? *reinterpret_cast<const float4*>(args.exp_avg_sq + 4 * oq) : float4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < NMR; ++i) {
      const int q = slotq(i);
      const bool own = q >= 0;
      mreg[i] = own ? *reinterpret_cast<const float4*>(args.exp_avg + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
      vreg[i] = own ? *reinterpret_cast<const float4*>(args.exp_avg_sq + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float step0 = args.adam_step[0];
  if (t < 24) reinterpret_cast<unsigned long long*>(hdr + 16)[t] = 0ull;
  if (t == 0) {   // 1 / B of a full and of the last minibatch (read per step from LDS, below)
    const int64_t blast = std::min<int64_t>(args.mb, args.N - (int64_t)(args.nb - 1) * args.mb);
    hdr[117] = 1.0f / (float)args.mb;
    hdr[118] = 1.0f / (float)std::max<int64_t>(blast, 1);
  }
  for (int k = t; k < Lp + 4; k += SPL_NT) Ga[k] = 0.0f;   // entries no tile writes stay 0 for good
  __syncthreads();

  unsigned long long* const pts = reinterpret_cast<unsigned long long*>(hdr + 64);
  if (g == 0 && t == 0) {
    for (int i = 0; i < 7; ++i) pts[i] = 0ull;
    pts[7] = __builtin_amdgcn_s_memrealtime();
    pts[8] = pts[7];
    pts[9] = __builtin_amdgcn_s_memtime();
  }
  auto mark = [&](int i) {
    if (args.profile && g == 0 && t == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      pts[i] += now - pts[7];
      pts[7] = now;
    }
  };
  unsigned long long* const tm = reinterpret_cast<unsigned long long*>(hdr + 16);
  const UpdSub subm{(args.profile && g == 0) ? tm + 8 : nullptr, pts + 7};
  const int R = args.R;   // == UPD_RT: one tile per workgroup and step
  // The loop top is on every step's critical path (AdamW -> next tile), so the per-step scalars
  // and the tile loads' addresses are loop-invariant pieces plus a row base: minibatch j = s mod
  // nb advanced by one per step, B (and this workgroup's rows) of a full and of the last
  // minibatch, and each thread's input offsets fixed at the start (upd_tile_load's addresses,
  // less its per-step branching: 0.56 us from the AdamW barrier to the tile's start).
  constexpr int KSM = upd_ksm<KA>();
  const int nb = args.nb;
  // rows of minibatch jj (B <= 0: past this data-parallel rank's rows), this workgroup's share
  auto B_of = [&](int jj) { return (int)std::min<int64_t>(args.mb, args.N - (int64_t)jj * args.mb); };
  auto rows_of = [&](int B) { return args.profile == 2 ? 0 : std::max(0, std::min(R, B - gt * R)); };
  const int Blast = B_of(nb - 1);   // (one rank: the only minibatch short of mb)
  const float invB_full = 1.0f / (float)args.mb, invB_last = 1.0f / (float)std::max(Blast, 1);
  const int ll = t & 63, lx = ll & 15, lq = ll >> 4;
  int xo[KSM];
  unsigned okb = 0u;
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
    const int d = 4 * s + lq;
    xo[s] = lx * n.D + d;
    okb |= (s < ((n.D + 3) >> 2) && d < n.D) ? 1u << s : 0u;
  }
  const float* rb = nullptr;   // this thread's row-input column (act[k] / old_logp / adv / ret)
  int rst = 0, rr_ = 0;
  if (t < UPD_RT * UPD_RIN) {
    const int k = t % UPD_RIN, Aw = n.discrete ? 1 : n.A;
    rr_ = t / UPD_RIN;
    if (k < UPD_MAXA) { if (k < Aw) { rb = args.act + k; rst = Aw; } }
    else if (k == 8) { rb = args.old_logp; rst = 1; }
    else if (k == 9) { rb = args.adv; rst = 1; }
    else if (k == 10) { rb = args.ret; rst = 1; }
  }
  const float* const Sg = args.S;
  // the inputs of minibatch jj's tile gt (upd_tile_load<.., RAW>: dummy loads of S[0] where empty)
  auto tile_load = [&](int jj, int rc, UpdIn<KSM>& in) {
    const int64_t row0 = (int64_t)jj * args.mb + (int64_t)gt * R;
    const float* Sb = Sg + row0 * n.D;
    const bool rowok = lx < rc;
    const unsigned ok = rowok ? okb : 0u;
#pragma unroll
    for (int s = 0; s < KSM; ++s) in.xin[s] = *(((ok >> s) & 1u) ? Sb + xo[s] : Sg);
    const bool rv = rb != nullptr && rr_ < rc;
    in.rin = *(rv ? rb + (row0 + rr_) * rst : Sg);
    in.ok = ok | (rv ? 1u << 31 : 0u);
  };
  UpdIn<KSM> nin;
  tile_load(0, rows_of(B_of(0)), nin);
  const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_part2 = upd_rsrc(args.part2),
                               rs_red = upd_rsrc(args.red);
  const __amdgpu_buffer_rsrc_t rs_mypart = upd_rsrc(args.part + (size_t)gt * Qtot * 4);
  const bool direct = args.spl_direct != 0;
  // the dW1 quads of this role's head: [W1lo, W1hi); stored from registers when direct, so their
  // padding columns (64..67 of each row) are zeroed once here and never written again
  const int W1lo = n.w1[role].lds / 4, W1hi = (n.w1[role].lds + UPD_H * UPD_HS) / 4;
  if (direct) {
    for (int q = W1lo + t; q < W1hi; q += SPL_NT) st4_sc1(rs_mypart, (size_t)q * 4, float4{0.f, 0.f, 0.f, 0.f});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (WB) {
    // the per-wave publish never writes the W1 / W2 padding quads nor the loss quad's other
    // words: this workgroup's partial regions start at zero (drained before any publish)
    const float4 z = {0.f, 0.f, 0.f, 0.f};
    if (role == 0) {
      for (int q = t; q < QH; q += SPL_NT) st4_sc1(rs_part, ((size_t)gt * Qtot + q) * 4, z);
      if (t == 0) st4_sc1(rs_part, ((size_t)gt * Qtot + Qp) * 4, z);
    } else {
      for (int q = QH + t; q < Qp; q += SPL_NT) st4_sc1(rs_part, ((size_t)gt * Qtot + q) * 4, z);
      for (int q = t; q <= QT; q += SPL_NT) st4_sc1(rs_part2, ((size_t)gt * (QT + 1) + q) * 4, z);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float loss_last = 0.f;
  const SplSlice& slc = slc0;
  // WB: the trunk's forward of the NEXT step's tile runs inside this step's AdamW (right after
  // slot 0, which holds the wave's W0 block and γ0 / β0: spl_wb_quad), beside the other slots'
  // updates; the first step's here.  (Fs is free: its last reader, dW1, is behind the tile's
  // barriers; the next tile reads it after its barrier #0.)
  upd_v4 nxh0 = {0.f, 0.f, 0.f, 0.f};
  float nr0 = 0.f;
  if constexpr (WB) spl_trunk_fwd<KSM>(n, W, sc, upd_in_real(nin).xin, nxh0, nr0);
  // the AdamW arithmetic of one quad (the engine's 4-wave scalar form): clipped gradient g4 * c
  auto adamw_quad = [&](const float4 g4, float4& m4, float4& v4, float4& pw, float clipc) {
    const float step_size = s_adam[0];
    const float inv_bc2_sqrt = s_adam[1];
    const float decay = (float)(1.0 - (double)args.lr * (double)args.wd);
    const float b2 = (float)args.beta2;
    const float omb1 = (float)(1.0 - (double)args.beta1), omb2 = (float)(1.0 - (double)args.beta2);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gr = f4get(g4, e) * clipc;
      float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
      p = p * decay;
      m = fmaf(omb1, gr - m, m);
      v = fmaf(omb2 * gr, gr, v * b2);
      const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2_sqrt, args.eps);
      float rq = __builtin_amdgcn_rcpf(denom);
      rq = fmaf(rq, fmaf(-denom, rq, 1.0f), rq);
      p = fmaf(-step_size, m * rq, p);
      f4set(m4, e, m);
      f4set(v4, e, v);
      f4set(pw, e, p);
    }
  };
  float4 og = {0.f, 0.f, 0.f, 0.f}, onm = {0.f, 0.f, 0.f, 0.f}, onv = {0.f, 0.f, 0.f, 0.f};
  unsigned nclip = 0;   // OWN: clipped steps so far (counter C's target), the same on every workgroup
  int j = 0;   // s mod nb
  int Bj = B_of(0);
  for (int s = 0; s < args.total_steps; ++s) {
    const int jn = j == nb - 1 ? 0 : j + 1;
    const int Bn = B_of(jn);
    // (1 / B from LDS: as a loop-invariant register value the compiler re-derived the division
    // in the loop top, on every step's critical path)
    const float invB = DP ? args.inv_count[j] : hdr[Bj == args.mb ? 117 : 118];
    const int myrows = rows_of(Bj);
    // ---- phase A: this role's share of tile group gt's gradient ------------------------------
    // (the next step's prefetch stays here: issued during wait A instead, by the waves idle
    // while wave 0 polls, it made the tile 0.13 us shorter and wait A 0.35 us longer —
    // profiles/r06_prefetch_in_waitA_ab.txt)
    if (myrows > 0) {
      const UpdIn<KSM> cur = upd_in_real(nin);
      // prefetch the next step's tile under this one and the hand-offs
      tile_load(jn, rows_of(Bn), nin);
      spl_tile<KA, TW, WB>(n, args, role, W, Ga, sc, cur, myrows, invB, tm, direct, rs_mypart, nxh0, nr0);
    } else {
      for (int k = t; k < Lp + 4; k += SPL_NT) Ga[k] = 0.0f;
      tile_load(jn, rows_of(Bn), nin);
    }
    j = jn;
    Bj = Bn;
    // (direct and rows this step: the dW1 quads are in the partial already; with no rows they
    // are published from the zeroed image like the rest)
    const bool skip = direct && myrows > 0;
    auto pub = [&](int q) {
      if (!(skip && q >= W1lo && q < W1hi))
        st4_sc1(rs_part, ((size_t)gt * Qtot + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
    };
    if (WB && myrows > 0) {
      // WB: each wave publishes its own list from the image entries it wrote itself (no
      // workgroup barrier in front); the loss words from waves 2 (k = role) and 3 (k = 2, actor)
      upd_wave_sync();
      mark(0);   // phase A compute (wave 0)
#pragma unroll
      for (int i = 0; i < SPL_WBQ; ++i) {
        const int q = wq[i];
        if (q >= 0 && !(skip && q >= W1lo && q < W1hi)) {
          const float4 v = *reinterpret_cast<const float4*>(Ga + 4 * q);
          if (role == 1 && q < QT) st4_sc1(rs_part2, ((size_t)gt * (QT + 1) + q) * 4, v);
          else st4_sc1(rs_part, ((size_t)gt * Qtot + q) * 4, v);
        }
      }
      const int w = t >> 6;
      if ((t & 63) == 0 && (w == 2 || (w == 3 && role == 0))) {
        const int k = w == 3 ? 2 : role;
        if (role == 0) st1_sc1(rs_part, (int)(((size_t)gt * Qtot + Qp) * 4) + k, Ga[Lp + k]);
        else st1_sc1(rs_part2, (int)(((size_t)gt * (QT + 1) + QT) * 4) + k, Ga[Lp + k]);
      }
    } else if (role == 0) {
      __syncthreads();
      mark(0);   // phase A compute
      const int qe = QH;   // trunk + head 0
      for (int q = t; q < qe; q += SPL_NT) pub(q);
      if (t == 0) st4_sc1(rs_part, ((size_t)gt * Qtot + Qp) * 4, *reinterpret_cast<const float4*>(Ga + Lp));
    } else {
      __syncthreads();
      mark(0);   // phase A compute
      for (int q = QH + t; q < Qp; q += SPL_NT) pub(q);
      for (int q = t; q < QT; q += SPL_NT)
        st4_sc1(rs_part2, ((size_t)gt * (QT + 1) + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
      if (t == 0) st4_sc1(rs_part2, ((size_t)gt * (QT + 1) + QT) * 4, *reinterpret_cast<const float4*>(Ga + Lp));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    mark(1);   // publish
    const bool skew = args.profile && (s & 15) == 0;
    if (t < 64) {
      if (skew && t == 0) spl_prof_stamp(args, 0, g);
      if (t == 0) upd_arrive(args.ctr, UPD_CTR_A, g);
      const bool ok = spl_wait(args, UPD_CTR_A, (unsigned)G * (unsigned)(s + 1));
      if (t == 0) *s_abort = ok ? 0 : 1;
    } else {
      if (t == 64) {
        const double tstep = (double)step0 + (double)(s + 1);
        const double bc1 = 1.0 - pow((double)args.beta1, tstep);
        const double bc2 = 1.0 - pow((double)args.beta2, tstep);
        s_adam[0] = (float)((double)args.lr / bc1);
        s_adam[1] = (float)(1.0 / sqrt(bc2));
      }
    }
    __syncthreads();
    if (*s_abort) return;
    mark(2);   // wait A
    if (skew && g == 0) {
      if (t < 64) spl_prof_skew(args, 0, G, Gt, tm);
      __syncthreads();
      if (t == 0) pts[7] = __builtin_amdgcn_s_memrealtime();   // (the read-back is no phase's)
    }
    // ---- phase B ---------------------------------------------------------------------------
    {
      const unsigned long long gstep = args.dp_seq0 + (unsigned long long)s;
      const int par = (int)(gstep & 1ull);
      spl_slice_reduce<SPL_NT>(rs_part, rs_part2, DP ? upd_rsrc(args.xbuf_self + (size_t)par * Qtot * 4) : rs_red,
                               Qtot, Qp, QT, slc, Gt, scratch, DP, subm, args, par, OWN ? &og : nullptr,
                               (!DP && !OWN && (WB || args.spl_pieces)) ? args.sq : nullptr);
      if constexpr (OWN) {
        // the owner's speculative AdamW (clip coefficient 1) on its quad; the new weights go out
        // in place of the gradient, with this wave's piece of the squared norm
        float sqv = 0.f;
        if (oq >= 0) {
          float4 pw = *reinterpret_cast<const float4*>(W + 4 * oq);
          onm = mreg[0];
          onv = vreg[0];
          adamw_quad(og, onm, onv, pw, 1.0f);
          st4_sc1(rs_red, (size_t)oq * 4, pw);
          sqv = (og.x * og.x + og.y * og.y) + (og.z * og.z + og.w * og.w);
        }
        sqv = wave_sum_f32_to63(sqv);
        if ((t & 63) == 63) st_sc1f(args.sq + (size_t)g * TW + (t >> 6), sqv);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (DP) {
        const int qlo = slc.qlo, qhi = slc.qhi;
        float* const pcs = (WB || args.spl_pieces) ? args.sq : nullptr;
        if (!(args.dp_push ? upd_dp_union_slice_push(args, rs_red, Qtot, g, gstep, par, s_abort, qlo, qhi, pcs)
                           : upd_dp_union_slice(args, rs_red, Qtot, g, G, gstep, par, s_abort, qlo, qhi, pcs)))
          return;
      }
    }
    mark(3);   // slice reduce
    if (t < 64) {
      if (args.profile && (s & 15) == 8 && t == 0) spl_prof_stamp(args, 1, g);
      if (t == 0) upd_arrive(args.ctr, UPD_CTR_B, g);
      const bool ok = spl_wait(args, UPD_CTR_B, (unsigned)Gs * (unsigned)(s + 1));
      if (t == 0) *s_abort = ok ? 0 : 1;
    }
    __syncthreads();
    if (*s_abort) return;
    mark(4);   // wait B
    if (args.profile && (s & 15) == 8 && g == 0) {   // (not A's sampled steps: its read-back delays g 0)
      if (t < 64) spl_prof_skew(args, 1, Gs, Gt, tm);
      __syncthreads();
      if (t == 0) pts[7] = __builtin_amdgcn_s_memrealtime();
    }
    // ---- phase C: the norm in the canonical order, then AdamW on the owned quads -------------
    float4 gq[WB ? SPL_WBQ : NQC];
    float clipc;
    {
      const bool pcs = WB || (!OWN && args.spl_pieces);   // (WB: always the pieces)
      float tot = 0.f;
      if (pcs) {
        // the norm from the pieces, loaded FIRST: every wave sums all of them itself (lane l:
        // pieces 4 l .. 4 l + 3 of each 256-piece chunk, chunk by chunk, then the DPP tree; the
        // same order and bits in every wave of every workgroup), so no workgroup barrier holds
        // AdamW until the whole gradient has landed: slot i's update waits for slot i's loads only
        const int nch = (Qp + SPL_CQ - 1) / SPL_CQ;   // <= 1,024 (NQC <= 10 at 4 waves)
        const __amdgpu_buffer_rsrc_t rs_sq = upd_rsrc(args.sq);
        const int l = t & 63;
        float4 pc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (256 * c < nch) pc[c] = ld4_sc1_so(rs_sq, 16u * (unsigned)l, 1024u * (unsigned)c);
        if constexpr (WB) {
          // this wave's block list (past its end: quad 0, unused)
#pragma unroll
          for (int i = 0; i < SPL_WBQ; ++i)
            gq[i] = ld4_sc1_so(rs_red, 16u * (unsigned)(wq[i] >= 0 ? wq[i] : 0), 0u);
        } else {
          // this role's slots (uniform per workgroup: a slot any of its quads is owned in)
#pragma unroll
          for (int i = 0; i < NQC; ++i)
            if (i * SPL_NT < Qp && (role == 0 ? i * SPL_NT < QH : (i * SPL_NT < QT || (i + 1) * SPL_NT > QH)))
              gq[i] = ld4_sc1_so(rs_red, 16u * (unsigned)t, 16u * (unsigned)(i * SPL_NT));
        }
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = 256 * c + 4 * l;
          if (256 * c < nch && k < nch)
            acc += ((pc[c].x + (k + 1 < nch ? pc[c].y : 0.f)) + ((k + 2 < nch ? pc[c].z : 0.f) + (k + 3 < nch ? pc[c].w : 0.f)));
        }
        acc = wave_sum_f32_to63(acc);
        tot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), 63));
        subm.mark(2);   // thread 0's pieces landed
      } else if constexpr (!WB) {
#pragma unroll
        for (int i = 0; i < NQC; ++i)
          if (i * SPL_NT < Qp) gq[i] = ld4_sc1_so(rs_red, 16u * (unsigned)t, 16u * (unsigned)(i * SPL_NT));
      }
      if (pcs) {
      } else if constexpr (OWN) {
        // gq: the NEW weights; the norm from the G x TW pieces, in one fixed order everywhere
        // (lane l: pieces 4 l .. 4 l + 3 of each 256-piece chunk, every chunk's load issued first)
        const int l = t & 63, npc = G * TW;
        const __amdgpu_buffer_rsrc_t rs_sq = upd_rsrc(args.sq);
        float4 pc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (256 * c < npc) pc[c] = ld4_sc1_so(rs_sq, 16u * (unsigned)l, 1024u * (unsigned)c);
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (256 * c < npc && 256 * c + 4 * l < npc) v += (pc[c].x + pc[c].y) + (pc[c].z + pc[c].w);
        v = wave_sum_f32_to63(v);
        tot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
        subm.mark(2);   // thread 0's weight quads and the pieces landed
      } else if constexpr (!WB) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NQC; ++i)
          if (i * SPL_NT < Qp && t + i * SPL_NT < Qp)
            acc += (gq[i].x * gq[i].x + gq[i].y * gq[i].y) + (gq[i].z * gq[i].z + gq[i].w * gq[i].w);
        subm.mark(2);   // thread 0's gradient quads landed
        acc = wave_sum_f32_to63(acc);
        float* s_nrm = hdr + 96;
        if ((t & 63) == 63) s_nrm[t >> 6] = acc;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < TW; ++w) tot += s_nrm[w];
      }
      const float coef = args.max_norm / (sqrtf(tot) + 1e-6f);
      clipc = coef < 1.0f ? coef : 1.0f;
      if (args.profile && g == 0 && t == 0 && coef < 1.0f) tm[20] += 1ull;
      if (g == 0 && t == 0 && s + 1 == args.total_steps) {
        const float4 lpq = ld4_sc1(rs_red, (size_t)Qp * 4);
        loss_last = lpq.x * invB + args.vf_coef * (lpq.y * invB) - args.ent_coef * (lpq.z * invB);
      }
    }
    mark(5);   // norm + loss
    if constexpr (OWN) {
      if (clipc < 1.0f) {
        // clip_grad_norm_ scaled this step (rare): the owners redo their quads with the true
        // coefficient from the kept gradient / moments and the LDS weights (not yet replaced),
        // publish them in red_c, and one more hand-off (counter C) precedes the weight load
        if (oq >= 0) {
          float4 pw = *reinterpret_cast<const float4*>(W + 4 * oq);
          onm = mreg[0];
          onv = vreg[0];
          adamw_quad(og, onm, onv, pw, clipc);
          st4_sc1(upd_rsrc(args.red + (size_t)Qtot * 4), (size_t)oq * 4, pw);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ++nclip;
        if (t < 64) {
          if (t == 0) upd_arrive(args.ctr, UPD_CTR_C, g);
          const bool ok = upd_wait_sharded(args.ctr, UPD_CTR_C, (unsigned)G * nclip);
          if (t == 0) *s_abort = ok ? 0 : 1;
        }
        __syncthreads();
        if (*s_abort) return;
        const __amdgpu_buffer_rsrc_t rs_redc = upd_rsrc(args.red + (size_t)Qtot * 4);
#pragma unroll
        for (int i = 0; i < NQC; ++i)
          if (i * SPL_NT < Qp) gq[i] = ld4_sc1_so(rs_redc, 16u * (unsigned)t, 16u * (unsigned)(i * SPL_NT));
      }
      mreg[0] = onm;   // commit the owner's moments
      vreg[0] = onv;
#pragma unroll
      for (int i = 0; i < NQC; ++i)
        if (i * SPL_NT < Qp && t + i * SPL_NT < Qp)
          *reinterpret_cast<float4*>(W + 4 * (t + i * SPL_NT)) = gq[i];
    } else {
      const float step_size = s_adam[0];
      const float inv_bc2_sqrt = s_adam[1];
      const float decay = (float)(1.0 - (double)args.lr * (double)args.wd);
      const float b2 = (float)args.beta2;
      const float omb1 = (float)(1.0 - (double)args.beta1), omb2 = (float)(1.0 - (double)args.beta2);
#pragma unroll
      for (int i = 0; i < NMR; ++i) {
        const int q = slotq(i);
        if (q >= 0) {
          float4 pw = *reinterpret_cast<float4*>(W + 4 * q);
          float4 m4 = mreg[i], v4 = vreg[i];
          const float4 g4 = gq[i];
          // the engine's AdamW arithmetic (ppo_update_body, the 4-wave scalar form; hipcc pairs
          // the elements into packed-f32 instructions itself)
          {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gr = f4get(g4, e) * clipc;
            float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
            p = p * decay;
            m = fmaf(omb1, gr - m, m);
            v = fmaf(omb2 * gr, gr, v * b2);
            const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2_sqrt, args.eps);
            float rq = __builtin_amdgcn_rcpf(denom);
            rq = fmaf(rq, fmaf(-denom, rq, 1.0f), rq);
            p = fmaf(-step_size, m * rq, p);
            f4set(m4, e, m);
            f4set(v4, e, v);
            f4set(pw, e, p);
          }
          }
          mreg[i] = m4;
          vreg[i] = v4;
          *reinterpret_cast<float4*>(W + 4 * q) = pw;
        }
        if constexpr (WB) {
          if (i == 0) {   // slot 0 holds the trunk forward's parameters (this wave's own writes)
            upd_wave_sync();
            spl_trunk_fwd<KSM>(n, W, sc, upd_in_real(nin).xin, nxh0, nr0);
          }
        }
      }
    }
    // (WB: no barrier — each wave updated exactly the parameters its next forward reads before
    // the tile's barrier #0, spl_wb_quad)
    if constexpr (!WB) __syncthreads();
    mark(6);   // AdamW (OWN: the new weights into LDS)
  }
  // ---- write back: role 0's first workgroup the trunk + head 0, role 1's the critic head (OWN:
  //      every owner its slice quad) ------------------------------------------------------------
  if constexpr (OWN) {
    if (oq >= 0) {
      *reinterpret_cast<float4*>(args.params + 4 * oq) = *reinterpret_cast<const float4*>(W + 4 * oq);
      *reinterpret_cast<float4*>(args.exp_avg + 4 * oq) = mreg[0];
      *reinterpret_cast<float4*>(args.exp_avg_sq + 4 * oq) = vreg[0];
    }
  }
  if (gt == 0) {
    if constexpr (!OWN) {
      for (int i = 0; i < NMR; ++i) {
        const int q = slotq(i);
        if (q >= 0 && (role == 0 ? q < QH : q >= QH)) {
          *reinterpret_cast<float4*>(args.params + 4 * q) = *reinterpret_cast<const float4*>(W + 4 * q);
          *reinterpret_cast<float4*>(args.exp_avg + 4 * q) = mreg[i];
          *reinterpret_cast<float4*>(args.exp_avg_sq + 4 * q) = vreg[i];
        }
      }
    }
    if (g == 0 && t == 0) {
      for (int i = 0; i < 7; ++i) args.prof[i] = pts[i];
      args.prof[7] = (unsigned long long)args.total_steps;
      args.prof[30] = __builtin_amdgcn_s_memrealtime() - pts[8];
      args.prof[31] = __builtin_amdgcn_s_memtime() - pts[9];
      for (int i = 0; i < 22; ++i) args.prof[8 + i] = reinterpret_cast<unsigned long long*>(hdr + 16)[i];
      args.adam_step[0] = step0 + (float)args.total_steps;
      if (args.loss_out) args.loss_out[0] = loss_last;
    }
  }
}

template <int NQC, int KA, int KDIM, bool DP = false, int TW = 4, bool OWN = false>
__global__ __launch_bounds__(64 * TW, 1) void ppo_update_split_kernel(UpdArgs args) {
  constexpr UpdNet N = upd_make(KDIM, KA, 1);
  ppo_split_body<NQC, KA, DP, TW, OWN>(N, args);
}
