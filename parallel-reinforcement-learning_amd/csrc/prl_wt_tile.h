// prl_wt_tile.h — included by prl_ppo_update.hip inside namespace prl (uses its Upd* types and helpers).
#pragma once
// ---- the wave-per-tile throughput form (WT, TPM = 2) -------------------------------------------
// For many tiles per workgroup and step (mini_batch >= 8,192; C2's second row, C3): the four
// waves of a workgroup (one per SIMD, 512 registers each) run WHOLE 16-row tiles independently —
// trunk, every head, output layer, loss and the whole backward for all 64 channels — with no
// workgroup barrier inside a tile.  Each wave accumulates its tiles' gradient in its own registers
// (dW1 of every head as 16 MFMA accumulators per head, MFMA-resident), and the four waves' sums
// meet once per step in an LDS image (wave order 0..3, fixed: deterministic).  The latency / TP
// forms split one tile over 8 waves with two workgroup barriers per tile, recompute the per-row
// loss in every wave, and spend ~72 % of their wave-cycles waiting (SQ counters,
// profiles/r04_tp_engine_pmc.json); here a wave has 4 independent accumulator chains per layer,
// and one wave per SIMD keeps the MFMA pipe fed.
//
// MFMA orientation as in the rest of the engine: v_mfma_f32_16x16x4_f32, C[m][n] at lane (x = n,
// q) register i = C[4q + i][x]; activations are C fragments [channel][row] (lane (row x, q) holds
// channels 16b + 4q + i of block b) and feed the next layer's B operand with the K order permuted
// (k-step (kb, i) <-> channel 16 kb + 4 q + i).  Contractions over rows (the weight gradients)
// read row-major copies from the wave's LDS scratch.  Specialised shapes only (CartPole: discrete,
// 2 actions; Pendulum: continuous, 1 action): one action column, nout <= 4 (all of a row's
// outputs in lane (row, q = 0)), D <= 16.

constexpr int WT_XS = 16;   // row stride of the wave's input copy [16][16]

// floats of one wave's scratch: Xs [16][16] | Fs [16][ZS] | Rin [16][4] | dOs [16][16] |
// Hs [nh][16][ZS] (a head's G, then its dZ; head 0's also dH0)
__host__ __device__ constexpr int upd_wt_wave_floats(int nh) {
  return 16 * WT_XS + 16 * UPD_ZS + 16 * 4 + 16 * 16 + nh * 16 * UPD_ZS;
}
// the workgroup's scratch region (the four waves' scratch; the step's gradient image Ga aliases it
// after the tiles)
__host__ __device__ constexpr int upd_wt_scratch_floats(const UpdNet& n) {
  const int a = 4 * upd_wt_wave_floats(n.nh), b = n.Lp + 4;
  return ((a > b ? a : b) + 3) & ~3;
}

template <int NH>
struct UpdWtGrad {
  upd_v4 w1[NH][16];   // dW1_h block (ob, ib): [16 ob + 4q + i][16 ib + x]
  upd_v4 w2[NH][4];    // dW2_h block ib: [4q + i][16 ib + x] (rows < out_h meaningful)
  upd_v4 w0[4];        // dW0 block b: [16 b + 4q + i][x] (x < D meaningful)
  float cg[1 + NH], cb[1 + NH];   // GN gamma / beta sums of layer L (trunk, heads), channel
                                  // 16 (x >> 2) + 4 q + (x & 3) of lane (x, q)
  float bias[4], loss[3];         // lane (x, q = 0): its rows' dO[j] / loss terms (summed at the end)
  __device__ void zero() {
    const upd_v4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < NH; ++h) {
#pragma unroll
      for (int k = 0; k < 16; ++k) w1[h][k] = z;
#pragma unroll
      for (int k = 0; k < 4; ++k) w2[h][k] = z;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) w0[k] = z;
#pragma unroll
    for (int k = 0; k < 1 + NH; ++k) cg[k] = cb[k] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) bias[k] = 0.f;
    loss[0] = loss[1] = loss[2] = 0.f;
  }
};

// sums over the tile's rows (DPP row of 16 lanes) of a channel-quad fragment; lane x keeps the
// sum of register i of block b where x == 4 b + i
__device__ inline void upd_wt_colsum(upd_v4 v, int b, float& acc) {
  const int x = threadIdx.x & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float s = upd_rsum16(v[i]);
    acc += (x == 4 * b + i) ? s : 0.f;
  }
}

// One wave's tile inputs (loaded ahead, UpdIn's selected-address form): lane (row x, q): X[row
// x][4 s + q] for s < KS, and field q of the row record (0 action, 1 old_logp, 2 adv, 3 ret).
template <int KSM>
__device__ inline void upd_wt_load(const UpdNet& n, const UpdArgs& args, int64_t row0, int rc,
                                   UpdIn<KSM>& in) {
  const int l = threadIdx.x & 63, x = l & 15, q = l >> 4;
  const int D = n.D, KS = (D + 3) >> 2;
  const bool rowok = x < rc;
  unsigned ok = 0u;
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
    const int d = 4 * s + q;
    const bool v = s < KS && rowok && d < D;
    in.xin[s] = *(v ? args.S + (row0 + x) * D + d : args.S);
    ok |= v ? 1u << s : 0u;
  }
  const float* src = q == 0 ? args.act : (q == 1 ? args.old_logp : (q == 2 ? args.adv : args.ret));
  in.rin = *(rowok ? src + row0 + x : args.S);   // (one action column: act is [N] or [N][1])
  ok |= rowok ? 1u << 31 : 0u;
  in.ok = ok;
}

template <int KD, int KA>
__device__ void upd_wt_tile(const UpdNet& n, const UpdArgs& args, const float* W, float* wsc,
                            const UpdIn<upd_ksm<KA>()>& in_raw, int rc, float invB,
                            UpdWtGrad<upd_kd_discrete(KD) ? 2 : 3>& gr) {
  constexpr int KSM = upd_ksm<KA>();
  constexpr int NH = upd_kd_discrete(KD) ? 2 : 3;
  const int l = threadIdx.x & 63, x = l & 15, q = l >> 4;
  const int D = n.D, KS = (D + 3) >> 2;
  float* Xs = wsc;
  float* Fs = Xs + 16 * WT_XS;
  float* Rin = Fs + 16 * UPD_ZS;
  float* dOs = Rin + 16 * 4;
  float* Hs = dOs + 16 * 16;   // [NH][16][ZS]
  const UpdIn<KSM> in = upd_in_real(in_raw);
  // ---- inputs -> LDS (row-major X for dW0, row records for the loss lanes)
#pragma unroll
  for (int s = 0; s < KSM; ++s)
    if (s < KS) Xs[x * WT_XS + 4 * s + q] = in.xin[s];
  Rin[x * 4 + q] = in.rin;
  // ---- trunk: 4 channel blocks
  upd_v4 F[4], xh0[4];
  float r0[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    upd_v4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wr = W + n.w0.lds + (16 * b + x) * n.w0.stride;
#pragma unroll
    for (int s = 0; s < KSM; ++s) {
      if (s < KS) {
        const int d = 4 * s + q;
        acc = upd_mma(d < D ? wr[d] : 0.0f, in.xin[s], acc);
      }
    }
    upd_gn_fwd_frag(acc, upd_ld4(W + n.g0.lds + 16 * b + 4 * q), upd_ld4(W + n.b0.lds + 16 * b + 4 * q),
                    xh0[b], r0[b], F[b]);
    upd_st4(Fs + x * UPD_ZS + 16 * b + 4 * q, F[b]);
  }
  // ---- heads (4 independent block chains each), their G row-major into Hs[h], output layer
  upd_v4 xh[NH][4];
  float rh[NH][4];
  upd_v4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const UpdHead hi = upd_head_info(n, h);
    upd_v4 z[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) z[ob] = upd_v4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      upd_v4 wa[4];
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) wa[ob] = upd_ld4(W + hi.w1 + (16 * ob + x) * UPD_HS + 16 * kb + 4 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) z[ob] = upd_mma(wa[ob][i], F[kb][i], z[ob]);
    }
    upd_v4 G[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      upd_gn_fwd_frag(z[ob], upd_ld4(W + hi.g1 + 16 * ob + 4 * q), upd_ld4(W + hi.b1 + 16 * ob + 4 * q),
                      xh[h][ob], rh[h][ob], G[ob]);
      upd_st4(Hs + h * 16 * UPD_ZS + x * UPD_ZS + 16 * ob + 4 * q, G[ob]);
    }
    // output layer: O^T[j][row] += W2_h[j - oc][k] G[row][k] (A rows j of this head, else 0)
    const bool mine = x >= hi.oc && x < hi.oc + hi.no;
    const float* w2r = W + hi.w2 + (mine ? x - hi.oc : 0) * UPD_HS;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const upd_v4 wv = mine ? upd_ld4(w2r + 16 * kb + 4 * q) : upd_v4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (kb & 1) o1 = upd_mma(wv[i], G[kb][i], o1);
        else o0 = upd_mma(wv[i], G[kb][i], o0);
      }
    }
  }
  // ---- loss of row x on lanes q == 0: outputs j = 0..3 are this lane's registers
  upd_wave_sync();   // Rin
  float dO[UPD_MAXO];
  float lp[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < UPD_MAXO; ++j) dO[j] = 0.f;
  if (q == 0) {
    float O[UPD_MAXO];
#pragma unroll
    for (int j = 0; j < UPD_MAXO; ++j) O[j] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) O[j] = j < n.nout ? o0[j] + o1[j] + W[upd_bias_of(n, j)] : 0.f;
    if (x < rc) {
      const upd_v4 r4 = upd_ld4(Rin + x * 4);
      float rin[UPD_RIN];
#pragma unroll
      for (int k = 0; k < UPD_RIN; ++k) rin[k] = 0.f;
      rin[0] = r4[0];
      rin[8] = r4[1];
      rin[9] = r4[2];
      rin[10] = r4[3];
      upd_row_loss<KD, KA>(n, O, rin, invB, args.clip, args.vf_coef, dO, lp);
    }
    upd_st4(dOs + x * 16, upd_v4{dO[0], dO[1], dO[2], dO[3]});
#pragma unroll
    for (int j = 0; j < 4; ++j) gr.bias[j] += dO[j];
#pragma unroll
    for (int k = 0; k < 3; ++k) gr.loss[k] += lp[k];
  }
  upd_wave_sync();   // dOs, Hs (G)
  // ---- backward: the trunk's B fragments for every head's dW1 (rows x channels)
  float fb[4][4];
#pragma unroll
  for (int ib = 0; ib < 4; ++ib)
#pragma unroll
    for (int s = 0; s < 4; ++s) fb[ib][s] = Fs[(4 * s + q) * UPD_ZS + 16 * ib + x];
  upd_v4 dF[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) dF[b] = upd_v4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const UpdHead hi = upd_head_info(n, h);
    const int oc = hi.oc, no = hi.no;
    float* Hh = Hs + h * 16 * UPD_ZS;
    // dW2_h[j][16 ib + x] += sum_rows dO[row][oc + j] G_h[row][16 ib + x]
    float ad[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ad[s] = x < no ? dOs[(4 * s + q) * 16 + oc + x] : 0.f;
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        gr.w2[h][ib] = upd_mma(ad[s], Hh[(4 * s + q) * UPD_ZS + 16 * ib + x], gr.w2[h][ib]);
    // dG_h^T block ob = W2_h^T dO_h^T (K = the head's outputs), GroupNorm + SiLU backward
    upd_v4 dz[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      upd_v4 dg = {0.f, 0.f, 0.f, 0.f};
      const bool kq = q < no;   // one k-step: outputs <= 4
      dg = upd_mma(kq ? W[hi.w2 + q * UPD_HS + 16 * ob + x] : 0.f, kq ? dOs[x * 16 + oc + q] : 0.f, dg);
      upd_v4 dy;
      dz[ob] = upd_gn_bwd_frag(dg, xh[h][ob], upd_ld4(W + hi.g1 + 16 * ob + 4 * q),
                               upd_ld4(W + hi.b1 + 16 * ob + 4 * q), rh[h][ob], dy);
      upd_v4 dyx;
#pragma unroll
      for (int i = 0; i < 4; ++i) dyx[i] = dy[i] * xh[h][ob][i];
      upd_wt_colsum(dyx, ob, gr.cg[1 + h]);
      upd_wt_colsum(dy, ob, gr.cb[1 + h]);
    }
    upd_wave_sync();   // every lane has read G_h (dW2) before dZ_h overwrites it
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) upd_st4(Hh + x * UPD_ZS + 16 * ob + 4 * q, dz[ob]);
    upd_wave_sync();
    // dW1_h[16 ob + 4q + i][16 ib + x] += sum_rows dZ_h[row][16 ob + x'] F[row][16 ib + x]
    float az[4][4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int s = 0; s < 4; ++s) az[ob][s] = Hh[(4 * s + q) * UPD_ZS + 16 * ob + x];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
          gr.w1[h][4 * ob + ib] = upd_mma(az[ob][s], fb[ib][s], gr.w1[h][4 * ob + ib]);
    // dF^T block b += W1_h^T dZ_h^T (K = the head's channels, permuted: step (ob, i) <-> 16 ob + 4q + i)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          dF[b] = upd_mma(W[hi.w1 + (16 * ob + 4 * q + i) * UPD_HS + 16 * b + x], dz[ob][i], dF[b]);
  }
  // ---- trunk GroupNorm + SiLU backward -> dH0, then dW0 = dH0^T X (dH0 row-major via head 0's Hs)
  upd_v4 dH0[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    upd_v4 dy;
    dH0[b] = upd_gn_bwd_frag(dF[b], xh0[b], upd_ld4(W + n.g0.lds + 16 * b + 4 * q),
                             upd_ld4(W + n.b0.lds + 16 * b + 4 * q), r0[b], dy);
    upd_v4 dyx;
#pragma unroll
    for (int i = 0; i < 4; ++i) dyx[i] = dy[i] * xh0[b][i];
    upd_wt_colsum(dyx, b, gr.cg[0]);
    upd_wt_colsum(dy, b, gr.cb[0]);
  }
  upd_wave_sync();   // every lane has read head 0's dZ (dW1) before dH0 overwrites it
#pragma unroll
  for (int b = 0; b < 4; ++b) upd_st4(Hs + x * UPD_ZS + 16 * b + 4 * q, dH0[b]);
  upd_wave_sync();
  float xb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) xb[s] = x < D ? Xs[(4 * s + q) * WT_XS + x] : 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      gr.w0[b] = upd_mma(Hs[(4 * s + q) * UPD_ZS + 16 * b + x], xb[s], gr.w0[b]);
  upd_wave_sync();   // the next tile rewrites the scratch
}

// The wave's register gradient added into the step's LDS image Ga (zeroed by the caller), at the
// entries the latency form's image holds; the caller runs the four waves one after another.
template <int KD>
__device__ void upd_wt_grad_add(const UpdNet& n, UpdWtGrad<upd_kd_discrete(KD) ? 2 : 3>& gr, float* Ga) {
  constexpr int NH = upd_kd_discrete(KD) ? 2 : 3;
  const int l = threadIdx.x & 63, x = l & 15, q = l >> 4;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const UpdHead hi = upd_head_info(n, h);
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int ib = 0; ib < 4; ++ib)
#pragma unroll
        for (int i = 0; i < 4; ++i) Ga[hi.w1 + (16 * ob + 4 * q + i) * UPD_HS + 16 * ib + x] += gr.w1[h][4 * ob + ib][i];
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * q + i < hi.no) Ga[hi.w2 + (4 * q + i) * UPD_HS + 16 * ib + x] += gr.w2[h][ib][i];
    const int ch = 16 * (x >> 2) + 4 * q + (x & 3);
    Ga[hi.g1 + ch] += gr.cg[1 + h];
    Ga[hi.b1 + ch] += gr.cb[1 + h];
  }
  if (x < n.D) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) Ga[n.w0.lds + (16 * b + 4 * q + i) * n.w0.stride + x] += gr.w0[b][i];
  }
  {
    const int ch = 16 * (x >> 2) + 4 * q + (x & 3);
    Ga[n.g0.lds + ch] += gr.cg[0];
    Ga[n.b0.lds + ch] += gr.cb[0];
  }
  // output biases and loss terms: sums over the rows (lanes q == 0 hold them; others 0)
  float bs[4], ls[3];
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = upd_rsum16(q == 0 ? gr.bias[j] : 0.f);
#pragma unroll
  for (int k = 0; k < 3; ++k) ls[k] = upd_rsum16(q == 0 ? gr.loss[k] : 0.f);
  if (l == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < n.nout) Ga[upd_bias_of(n, j)] += bs[j];
#pragma unroll
    for (int k = 0; k < 3; ++k) Ga[n.Lp + k] += ls[k];
  }
}
