// tog_bwd_quad.hpp — the square-root backward pass of the convergence tail on four waves per trajectory.
//
// Reference: src/solvers/ilqr/backward_pass.jl:87-192 (_backwardpass_sqrt!, chol_plus, chol_minus).
//
// Round 4's three-wave variant ran Q.ux, then per released row of the new Q.xx factor one substitution
// step and one systolic chol_minus step on one wave (≈ 820 cycles a row against the QR's ≈ 650), so the
// chain waited on it (profiles/r4o_trio_sections_b1.txt); the two- and three-wave variants are retired
// (round 5). Here
//   wave A (QRs):   qr([Q.xx; S A]) releasing the factor's rows; as soon as K (B) and tmp1 (C) are out,
//                   the top rows Q.xx + tmp1 K of the S-update operand; after B2b its bottom rows
//                   tmp2 K and qr([Q.xx + tmp1 K; tmp2 K]) = S_k releasing S_k's rows
//   wave B (side):  Q.x/Q.u += [A B]'s, qr([Q.uu; S B]) (released to D), Quu_reg, cond, K, d, s_k, ΔV
//                   and the K/d stores (with C's Q.ux; K released to A); then the next knot's S_k A_{k-1}
//                   and S_k B_{k-1} from S_k's released rows
//   wave C (tmp1):  Q.ux += (S B)'(S A) (released to B), then tmp1 = Q.xx' \ Q.ux' one row per released
//                   row of the Q.xx factor, each row released to D (and to A)
//   wave D (chol):  chol_minus(Q.uu, tmp1), systolic step t as row t of tmp1 is released
// Two workgroup barriers per knot: B2b (tmp2, the verdict, the downdate's failure flag; all four waves
// restart or stop together) and B3 (S_k whole, S_k A_{k-1} and S_k B_{k-1} on the bus). Everything else
// passes through LDS tagged with the knot's sequence number (a release store after the data, an acquire
// load before the reads; see tag_store for why wavefront scope suffices and what the alternatives cost). Every
// value is computed by the same operations in the same order as the other backward kernels (and the
// oracle): the results are bit-identical.
#pragma once

namespace tog {

template <class M>
struct QuadLayout {  // doubles in the workgroup's LDS
  static constexpr int n = M::n, m = M::m;
  static constexpr int S = 0;                 // S_{k+1} (n*n, upper factor, zeros below) then s (n)
  static constexpr int QU = n * n + n;        // Q.uu factor (m*m, column-major; B -> C, B's s_k)
  static constexpr int TX = QU + m * m;       // S A (n*n, column c from lane c of wave B)
  static constexpr int TU = TX + n * n;       // S B (n*m, column c from lane c of wave B)
  static constexpr int QUX = TU + n * m;      // Q.ux (m*n, column c from lane c of wave C)
  static constexpr int KB = QUX + m * n;      // K (m*n, column c from lane c of wave B)
  static constexpr int RX = KB + m * n;       // the new Q.xx factor's released rows (n*n, A -> C)
  static constexpr int BA = RX + n * n;       // wave C's bus: tmp1 rows at +32, chol_minus output after
  static constexpr int BA_SIZE = 32 + n * m + 3 * m * m + 8;
  static constexpr int BB = BA + BA_SIZE;     // wave B's bus: :state B columns, cond scratch
  static constexpr int BB_SIZE = 2 * n * m + m * m + 8;
  static constexpr int FLAGS = BB + BB_SIZE;  // ints: [0] verdict (1 ok), [2] this knot's chol_minus failure (C -> all)
  static constexpr int QXT = FLAGS + 2;       // (S B)'(S A) for the next knot's Q.ux (m*n, column c from
                                              // lane c of wave B, summed as S's rows were released)
  static constexpr int PAD = QXT + m * n;     // 16 doubles: where the lanes past the team's columns store
                                              // their part of a released row (no per-lane branch)
  static constexpr int TAGS = PAD + 16;       // ints: S_k rows (n), Q.xx factor rows (n), Q.uu rows (m), Q.ux,
                                              // tmp1 rows (n), K
  static constexpr int NTAGS = 3 * n + m + 2;
  static constexpr int TOTAL = TAGS + (NTAGS + 1) / 2;
};

template <class M, int ALI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
k_bwd_quad(const DevProblem* P, DevBuffers Bf, int flags) {
  using Cfg = TeamCfg<M>;
  using D = QuadLayout<M>;
  constexpr bool SQRT = true, AL = (ALI & 1) != 0, TV = (ALI & 2) != 0;  // TV: a time-varying Objective
  constexpr int n = M::n, m = M::m, L = n + m, TEAM = Cfg::TEAM, NQ = nq_of<M>(), NE = ne_of<M>();
  static_assert(TEAM == 16 && m <= n && n + 1 <= 16, "quad kernel: 16-lane DPP rows");
  __shared__ double lds[D::TOTAL];
  __shared__ int kcnt[TEAM_MAX_KNOTS], knx[TEAM_MAX_KNOTS];
  const int wv = threadIdx.x >> 6;  // 0: QR wave A, 1: side wave B, 2: tmp1 wave C, 3: chol wave D (uniform)
  const int tl = threadIdx.x & 15;  // column of this lane (each DPP row computes the whole team)
  const long long b = traj_of_slot(Bf, blockIdx.x, P->B);
  if (b < 0) return;  // workgroup-uniform
  if (!Bf.st[b].active || Bf.st[b].ls_pend) return;
  BPROF_DECL
  const int N = P->N;
  if (AL) {
    for (int e = threadIdx.x; e < N; e += 256) {
      kcnt[e] = P->knot_cnt[e];
      knx[e] = P->knot_nx[e];
    }
  }
  int* tags = reinterpret_cast<int*>(lds + D::TAGS);
  int* rowf = tags;           // S_k's rows (A -> B)
  int* rxf = tags + n;        // the new Q.xx factor's rows (A -> C)
  int* qurf = tags + 2 * n;   // the Q.uu factor's rows (B -> D)
  int* quxf = qurf + m;       // Q.ux (C -> B)
  int* t1f = quxf + 1;        // tmp1's rows (C -> D, A)
  int* kf = t1f + n;          // K (B -> A)
  if (threadIdx.x < D::NTAGS) tags[threadIdx.x] = 0;
  __syncthreads();
  double* Sreg = lds + D::S;
  double* QU = lds + D::QU;
  double* TXb = lds + D::TX;
  double* QUXb = lds + D::QUX;
  double* KB = lds + D::KB;
  double* RX = lds + D::RX;
  double* busA = lds + D::BA;
  double* busB = lds + D::BB;
  double* pad = lds + D::PAD;
  double* QXT = lds + D::QXT;
  int* flg = reinterpret_cast<int*>(lds + D::FLAGS);
  constexpr int SOFF = n * n;
  constexpr int TB = 32;
  double* bus2 = busA + TB + n * m;
  const bool store_S = (flags & TOG_BP_STORE_S) && Bf.Sdbg;
  const bool state_reg = (P->o.bp_reg_type == 1);
  const double dt = P->dt;
  const double* ABg = Bf.AB + (size_t)b * (N - 1) * n * L;
  double* Kg = Bf.K + (size_t)b * (N - 1) * m * n;
  double* dg = Bf.d + (size_t)b * (N - 1) * m;
  double* Qs = Bf.Qscr + (size_t)b * N * NQ;
  const double* Eg = Bf.E + (size_t)b * N * NE;
  const bool colx = tl < n, colu = tl < m;
  const int c = colx ? tl : 0, cu = colu ? tl : 0;
  RegState s;  // (wave B's: ρ, dρ, flags)
  s.rho = Bf.st[b].rho;
  s.drho = Bf.st[b].drho;
  s.flags = Bf.st[b].flags;
  const double rho0 = s.rho, drho0 = s.drho;
  constexpr int RS = n + m;  // rows of the S-update operand
  // Registers carried across knots, one array shared by the wave roles (they are wave-exclusive; the
  // compiler cannot know it, so separate arrays would all stay live in every wave and spill):
  //   A: [0, n) the next knot's Q.xx column; [n, 2n) its Q.xx factor column, [2n, 2n+RS) the S-update
  //      operand column and [2n+RS, 2n+RS+m) K's column (within a knot)
  //   B: [0, n) A_k column, [n, 2n) B_k column, [2n, 3n) (S B) column, then Q.u (m), Q.uu column (m),
  //      the Q.x entry
  //   C: [0, m) the replayed Q.ux column, [m, 2m) H dt's column
  constexpr int NR = (2 * n + RS + m) > (3 * n + 2 * m + 1) ? (2 * n + RS + m) : (3 * n + 2 * m + 1);
  double R[NR];
#pragma unroll
  for (int i = 0; i < NR; i++) R[i] = 0.0;
  auto view = [&](auto off_c, auto len_c) -> double (&)[decltype(len_c)::value] {
    return *reinterpret_cast<double(*)[decltype(len_c)::value]>(R + decltype(off_c)::value);
  };
  using I0 = std::integral_constant<int, 0>;
  using In = std::integral_constant<int, n>;
  using I2n = std::integral_constant<int, 2 * n>;
  using I3n = std::integral_constant<int, 3 * n>;
  using Im = std::integral_constant<int, m>;
  using IRS = std::integral_constant<int, RS>;
  double(&Hdt)[m] = view(Im{}, Im{});  // (wave C) H dt's column, the Q.ux every non-replayed knot starts from
  if (wv == 2) {
#pragma unroll
    for (int i = 0; i < m; i++) Hdt[i] = P->H[i + m * c] * dt;
  }
  bool faithful = false;
  int kmin = N - 1, restarts = 0;
  double dV0 = 0.0, dV1 = 0.0;
  bool done = false;
  auto dense = [&](int k) { return knot_dense<SQRT, AL>(k, N, AL ? kcnt[k] : 0, AL ? knx[k] : 0); };
  int seq = 0;  // knot sequence number (every wave counts alike): the tags' value for this knot
  // The tag is a release store at wavefront scope, read with a workgroup-scope acquire. The release keeps
  // the compiler from moving the tagged data's stores after the tag; the cross-wave order then rests on
  // the hardware: the data and the tag are DS stores (no FLAT store in the kernel: every LDS access is a
  // DS instruction), and the LDS unit performs one wave's DS operations in issue order, so a consumer
  // that has read the tag and then reads the data sees the data. Measured alternatives
  // (profiles/r5_quad_tag_isa.txt, tools/quad_tag_isa.py): a workgroup-scope release adds an
  // s_waitcnt lgkmcnt(0) before each of the 33 tag stores; a bounded wait (a poll counter that flags an
  // error word or traps) grows the kernel from 10.6 k to 13-16 k instructions and the tail backward from
  // 0.886 to 0.96 ms per step (B = 1; whole solve 88.3 k -> 83.4 k it/s). The waits stay unbounded; a hang
  // is reported by the host watchdog of the blocking readbacks (tog_runtime.cpp wait_event) instead.
  // (Every lane stores the same tag: no exec-mask change splits the scheduling region.)
  auto tag_store = [&](int* t) { __hip_atomic_store(t, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WAVEFRONT); };
  auto tag_wait = [&](int* t) {
    while (__hip_atomic_load(t, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != seq) {
    }
  };
  // wave A: the Q.xx column entering knot kk's QR (the replayed one in faithful mode), loaded a knot ahead
  auto load_qxx = [&](int kk, double (&Qx)[n]) {
    if (faithful && kk >= kmin) {
      const double* qk = Qs + (size_t)kk * NQ;
#pragma unroll
      for (int i = 0; i < n; i++) Qx[i] = qk[n + m + i + n * c];
    } else if (dense(kk)) {
      const double* ek = Eg + (size_t)kk * NE;
#pragma unroll
      for (int i = 0; i < n; i++) Qx[i] = ek[n + m + m * m + i + n * c];
    } else {  // the stage cost's square-root factor (a time-varying Objective's knot kk)
      const double* cQ = TV ? cost_at<n, m>(P, kk).cQ : P->cQ;
#pragma unroll
      for (int i = 0; i < n; i++) Qx[i] = cQ[i + n * c];
    }
  };
  // wave B: knot kk's Q.x entry, Q.u and Q.uu column (the replayed ones in faithful mode), a knot ahead
  auto load_b = [&](int kk, double& xs, double (&qu)[m], double (&quu)[m]) {
    if (faithful && kk >= kmin) {
      const double* qk = Qs + (size_t)kk * NQ;
      xs = qk[c];
#pragma unroll
      for (int i = 0; i < m; i++) qu[i] = qk[n + i];
#pragma unroll
      for (int i = 0; i < m; i++) quu[i] = qk[n + m + n * n + i + m * cu];
    } else {
      const double* ek = Eg + (size_t)kk * NE;
      xs = ek[c];
#pragma unroll
      for (int i = 0; i < m; i++) qu[i] = ek[n + i];
#pragma unroll
      for (int i = 0; i < m; i++) quu[i] = ek[n + m + i + m * cu];
    }
  };
  // wave B: this lane's columns of A_kk and B_kk
  auto load_ab = [&](int kk, double (&Ac)[n], double (&Bc)[n]) {
    const double* abk = ABg + (size_t)kk * n * L;
#pragma unroll
    for (int i = 0; i < n; i++) {
      Ac[i] = abk[i + n * c];
      Bc[i] = abk[i + n * (n + cu)];
    }
  };
  // wave B: row i of tmp_x = S A and tmp_u = S B for this lane's columns, l ascending over the upper
  // factor's nonzero entries (the order of k_bwd_team's TRI_SA products: each entry is the same fma chain)
  // The next knot's tmp_u' tmp_x (backward_pass.jl:118) is accumulated here too, row i's terms as row i
  // comes: t[ii] = fma(tmp_u[i][ii], tmp_x[i][c], t[ii]), i ascending -- the order of the Q.ux sum.
  auto row_products = [&](auto ic, const double (&Ac)[n], const double (&Bc)[n], double (&Tb)[n], double (&tq)[m]) {
    constexpr int i = decltype(ic)::value;
    double sr[n - i];
#pragma unroll
    for (int l = i; l < n; l++) sr[l - i] = Sreg[i + n * l];
    double tx = 0.0, tu = 0.0;
#pragma unroll
    for (int l = i; l < n; l++) {
      tx = fma(sr[l - i], Ac[l], tx);
      tu = fma(sr[l - i], Bc[l], tu);
    }
    if (colx) TXb[i + n * tl] = tx;
    Tb[i] = tu;
    static_for<0, m>([&](auto iic) {
      constexpr int ii = decltype(iic)::value;
      tq[ii] = fma(row_bcast<ii>(tu), tx, tq[ii]);
    });
  };
  auto products_done = [&](const double (&tq)[m]) {
    if (colx) {
#pragma unroll
      for (int ii = 0; ii < m; ii++) QXT[ii + m * tl] = tq[ii];
    }
  };

  while (!done) {  // one attempt of the backward pass; a regularisation restart begins a new one
    if (wv == 0) {  // S[N] = Q[N] (backward_pass.jl:100-101), from the terminal expansion record
      const double* e = Eg + (size_t)(N - 1) * NE;
      double Qxc[n];
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] = e[n + m + m * m + i + n * c];
      const double Qxs = e[c];
      if (colx) {
#pragma unroll
        for (int i = 0; i < n; i++) Sreg[i + n * tl] = (i > tl) ? 0.0 : Qxc[i];
        Sreg[SOFF + tl] = Qxs;
      }
      if (store_S && colx) {
#pragma unroll
        for (int i = 0; i < n; i++) Bf.Sdbg[((size_t)b * N + (N - 1)) * n * n + i + n * tl] = Qxc[i];
        Bf.sdbg[((size_t)b * N + (N - 1)) * n + tl] = Qxs;
      }
    }
    __syncthreads();
    // carried across knots: wave A's next Q.xx column; wave B's A_k, B_k columns and S_{k+1} B_k
    double(&Qxn)[n] = view(I0{}, In{});
    double(&Ac)[n] = view(I0{}, In{});
    double(&Bc)[n] = view(In{}, In{});
    double(&Tb)[n] = view(I2n{}, In{});
    double(&Bqu)[m] = view(I3n{}, Im{});
    double(&Bquu)[m] = view(std::integral_constant<int, 3 * n + m>{}, Im{});
    double& Bxs = R[3 * n + 2 * m];
    double(&Cqr)[m] = view(I0{}, Im{});  // (wave C's replayed Q.ux)
    auto load_cqr = [&](int kk) {
      if (faithful && kk >= kmin) {
        const double* qk = Qs + (size_t)kk * NQ;
#pragma unroll
        for (int i = 0; i < m; i++) Cqr[i] = qk[n + m + n * n + m * m + i + m * c];
      }
    };
    if (wv == 2) load_cqr(N - 2);
    if (wv == 0) {
      load_qxx(N - 2, Qxn);
    } else if (wv == 1) {  // the first knot's products, from the whole terminal factor
      load_ab(N - 2, Ac, Bc);
      load_b(N - 2, Bxs, Bqu, Bquu);
      double tq[m] = {};
      static_for<0, n>([&](auto ic) { row_products(ic, Ac, Bc, Tb, tq); });
      products_done(tq);
    }
    __syncthreads();
    dV0 = 0.0;
    dV1 = 0.0;
    bool restart = false;
    for (int k = N - 2; k >= 0; k--) {
      seq++;
      const bool replay = faithful && k >= kmin;
      const double* q = Qs + (size_t)k * NQ;
      double(&Qxc)[n] = view(In{}, In{});  // (wave A's Q.xx factor column, kept for the S-update operands)
      double(&a2)[RS] = view(I2n{}, IRS{});  // (wave A's S-update operand column and K column, across B2b)
      double(&Kc)[m] = view(std::integral_constant<int, 2 * n + RS>{}, Im{});
      // ------------------------------------------------------------------ A: qr([Q.xx; S A]), rows released
      if (wv == 0) {
        {  // Q.xx <- qr([Q.xx; tmp_x]).R (backward_pass.jl:116), tmp_x = S A from wave B's bus
          double a[2 * n];
#pragma unroll
          for (int i = 0; i < n; i++) {
            a[i] = Qxn[i];
            a[n + i] = TXb[i + n * c];
          }
          DPROF(0);
          auto release = [&](auto jc, const double (&r)[2 * n]) {
            constexpr int j = decltype(jc)::value;
            *(colx ? RX + j + n * tl : pad + tl) = (j <= tl) ? r[j] : 0.0;
            tag_store(&rxf[j]);
          };
          team_qr<2 * n, n, n, TEAM, false>(a, 2 * n, tl, busA, release);
#pragma unroll
          for (int i = 0; i < n; i++) Qxc[i] = (i <= tl) ? a[i] : 0.0;
        }
        if (faithful && colx) {
#pragma unroll
          for (int i = 0; i < n; i++) Qs[(size_t)k * NQ + n + m + i + n * tl] = Qxc[i];
        }
        DPROF(1);
        // the top rows of the S-update operand, Q.xx + tmp1 K, as soon as K and all of tmp1 are out (a
        // knot that restarts leaves K unwritten: the rows are then discarded)
        tag_wait(kf);
        tag_wait(&t1f[n - 1]);
        DPROF(2);
#pragma unroll
        for (int i = 0; i < m; i++) Kc[i] = KB[i + m * c];
        {
          double v[n];
#pragma unroll
          for (int i = 0; i < n; i++) v[i] = 0.0;
#pragma unroll
          for (int l = 0; l < m; l++) {
#pragma unroll
            for (int i = 0; i < n; i++) v[i] = fma(busA[TB + i * m + l], Kc[l], v[i]);
            TEAM_FENCE();
          }
#pragma unroll
          for (int i = 0; i < n; i++) a2[i] = Qxc[i] + v[i];
        }
        DPROF(3);
      } else if (wv == 1) {
        // ---------------------------------------------------------------- B: Q.x, Q.u, qr([Q.uu; S B]), gains
        double Qxs = Bxs, Qu[m], Quuc[m], Quxc[m];
#pragma unroll
        for (int i = 0; i < m; i++) {
          Qu[i] = Bqu[i];
          Quuc[i] = Bquu[i];
        }
        {  // Q.uu <- qr([Q.uu; tmp_u]).R (backward_pass.jl:117), its rows released to wave D
          double a[m + n];
#pragma unroll
          for (int i = 0; i < m + n; i++) a[i] = (i < m) ? Quuc[i] : Tb[i - m];
          auto release = [&](auto jc, const double (&r)[m + n]) {
            constexpr int j = decltype(jc)::value;
            *(colu ? QU + j + m * tl : pad + tl) = (j <= tl) ? r[j] : 0.0;
            tag_store(&qurf[j]);
          };
          team_qr<m + n, m, m, TEAM, false>(a, m + n, tl, busB, release);
#pragma unroll
          for (int i = 0; i < m; i++) Quuc[i] = (i <= tl) ? a[i] : 0.0;
        }
        // Q.x += A's ; Q.u += B's (backward_pass.jl:112-113)
        {
          double t = 0.0;
#pragma unroll
          for (int l = 0; l < n; l++) t = fma(Ac[l], Sreg[SOFF + l], t);
          Qxs += t;
          double tu = 0.0;
#pragma unroll
          for (int l = 0; l < n; l++) tu = fma(Bc[l], Sreg[SOFF + l], tu);
          static_for<0, m>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            Qu[i] += row_bcast<i>(tu);
          });
        }
        if (faithful) {
          double* qq = Qs + (size_t)k * NQ;
          if (colx) qq[tl] = Qxs;
          if (colu) {
#pragma unroll
            for (int i = 0; i < m; i++) qq[n + m + n * n + i + m * tl] = Quuc[i];
          }
          if (tl == 0) {
#pragma unroll
            for (int i = 0; i < m; i++) qq[n + i] = Qu[i];
          }
        }
        DPROF(6);
        // regularise, test, gains (backward_pass.jl:120-145): Quu_reg = qr([Q.uu; sqrt(ρ) I]).R
        // (:control) or qr([Q.uu; sqrt(ρ) B]).R (:state)
        double F[m][m], rF[m];
        {
          const double sr = sqrt(s.rho);
          auto qr_reg = [&](auto& a) {
            constexpr int RR = sizeof(a) / sizeof(a[0]);
#pragma unroll
            for (int i = 0; i < RR; i++) {
              double v = 0.0;
              if (i < m) v = Quuc[i];
              else if (state_reg) v = sr * ABg[(size_t)k * n * L + n * (n + cu) + (i - m)];
              else if (i - m == tl) v = sr;
              a[i] = v;
            }
            team_qr<RR, m, m, TEAM, true>(a, RR, tl, busB);
            static_for<0, m>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
#pragma unroll
              for (int i = 0; i < m; i++) F[i][j] = (i <= j) ? row_bcast<j>(a[i]) : 0.0;
            });
          };
          if (state_reg) {
            double a[m + n];
            qr_reg(a);
          } else {
            double a[2 * m];
            qr_reg(a);
          }
        }
#pragma unroll
        for (int j = 0; j < m; j++) rF[j] = 1.0 / F[j][j];
        const bool ok = !cond_exceeds_team<m>(F, rF, 1e8, busB + 2 * n * m, tl);
        DPROF(7);
        tag_wait(quxf);
#pragma unroll
        for (int i = 0; i < m; i++) Quxc[i] = QUXb[i + m * c];
        DPROF(8);
        if (ok) {
          // right-hand side of this lane: Qux_reg column (state reg adds ρ B'A), or Q.u for lane n
          double col[m];
          if (state_reg) {  // (:state regularisation: the B columns on the bus)
            if (colu) {
              const double* bk = ABg + (size_t)k * n * L + n * (n + tl);
#pragma unroll
              for (int i = 0; i < n; i++) busB[n * m + i + n * tl] = bk[i];
            }
            team_sync();
          }
          if (colx) {
#pragma unroll
            for (int i = 0; i < m; i++) col[i] = Quxc[i];
            if (state_reg) {
              const double* ak = ABg + (size_t)k * n * L + n * c;
              double t[m];
#pragma unroll
              for (int i = 0; i < m; i++) t[i] = 0.0;
#pragma unroll 1
              for (int l = 0; l < n; l++) {
                const double a = ak[l];
#pragma unroll
                for (int i = 0; i < m; i++) t[i] = fma(busB[n * m + l + n * i], a, t[i]);
              }
#pragma unroll
              for (int i = 0; i < m; i++) col[i] += s.rho * t[i];
            }
          } else {
#pragma unroll
            for (int i = 0; i < m; i++) col[i] = Qu[i];
          }
          // K = -Quu_reg \ (Quu_reg' \ Qux_reg); contract v2: multiply by the diagonal reciprocals
#pragma unroll
          for (int j = 0; j < m; j++) {
            const double xj = col[j] * rF[j];
            col[j] = xj;
#pragma unroll
            for (int i = j + 1; i < m; i++) col[i] = fma(-F[j][i], xj, col[i]);
          }
#pragma unroll
          for (int j = m - 1; j >= 0; j--) {
            const double xj = col[j] * rF[j];
            col[j] = xj;
#pragma unroll
            for (int i = j - 1; i >= 0; i--) col[i] = fma(-F[i][j], xj, col[i]);
          }
          double Kc[m], d[m];
#pragma unroll
          for (int i = 0; i < m; i++) Kc[i] = -1.0 * col[i];
#pragma unroll
          for (int i = 0; i < m; i++) d[i] = row_bcast<n>(Kc[i]);
          if (colx) {
#pragma unroll
            for (int i = 0; i < m; i++) {
              Kg[(size_t)k * m * n + i + m * tl] = Kc[i];
              KB[i + m * tl] = Kc[i];
            }
          }
          if (tl == n) {
#pragma unroll
            for (int i = 0; i < m; i++) dg[(size_t)k * m + i] = Kc[i];
          }
          // s[c] = Q.x[c] + (K'Q.uu')(Q.uu d) + K'Q.u + Q.ux'd (backward_pass.jl:145)
          double Ud[m], KtU[m];
#pragma unroll
          for (int i = 0; i < m; i++) {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < m; l++) t = fma(QU[i + m * l], d[l], t);
            Ud[i] = t;
          }
#pragma unroll
          for (int j = 0; j < m; j++) {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < m; l++) t = fma(Kc[l], QU[j + m * l], t);
            KtU[j] = t;
          }
          double sown;
          {
            double a = 0.0, b2 = 0.0, c2 = 0.0;
#pragma unroll
            for (int l = 0; l < m; l++) {
              a = fma(KtU[l], Ud[l], a);
              b2 = fma(Kc[l], Qu[l], b2);
              c2 = fma(Quxc[l], d[l], c2);
            }
            sown = ((Qxs + a) + b2) + c2;
          }
          if (colx) Sreg[SOFF + tl] = sown;  // s_k (no wave reads s_{k+1} any more)
          if (store_S && colx) Bf.sdbg[((size_t)b * N + k) * n + tl] = sown;
          {  // ΔV += [d'Q.u, ½‖Q.uu d‖²] (backward_pass.jl:158-161)
            double a = 0.0, b2 = 0.0;
#pragma unroll
            for (int i = 0; i < m; i++) a = fma(d[i], Qu[i], a);
#pragma unroll
            for (int i = 0; i < m; i++) b2 = fma(Ud[i], Ud[i], b2);
            dV0 += a;
            dV1 += 0.5 * b2;
          }
        }
        if (threadIdx.x == 64) flg[0] = ok ? 1 : 0;
        tag_store(kf);
        DPROF(9);
      } else if (wv == 2) {
        // ---------------------------------------------------------------- C: Q.ux, tmp1
        double Quxc[m];
        if constexpr (TV) {  // knot k's H dt
          const double* Hk = cost_at<n, m>(P, k).H;
#pragma unroll
          for (int i = 0; i < m; i++) Quxc[i] = replay ? Cqr[i] : Hk[i + m * c] * dt;
        } else {
#pragma unroll
          for (int i = 0; i < m; i++) Quxc[i] = replay ? Cqr[i] : Hdt[i];  // sqrt AL adds no Q.ux term (A.5)
        }
        // Q.ux += tmp_u' tmp_x (backward_pass.jl:118), the sum wave B formed from S_{k+1}'s rows
#pragma unroll
        for (int i = 0; i < m; i++) Quxc[i] += QXT[i + m * c];
        if (colx) {
#pragma unroll
          for (int i = 0; i < m; i++) QUXb[i + m * tl] = Quxc[i];
        }
        tag_store(quxf);
        if (faithful && colx) {
#pragma unroll
          for (int i = 0; i < m; i++) Qs[(size_t)k * NQ + n + m + n * n + m * m + i + m * tl] = Quxc[i];
        }
        DPROF(13);
        // tmp1 = (Q.xx') \ Q.ux' by distributed forward substitution (lane i owns row i), step j as row j
        // of the factor is released; row j of tmp1 is final after step j and released in turn
        double t1[m];
#pragma unroll
        for (int i = 0; i < m; i++) t1[i] = Quxc[i];
        static_for<0, n>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          tag_wait(&rxf[j]);
          const double rj = RX[j + n * c];  // row j of the factor: R[j][j] on lane j, R[j][c] on lane c
          if (tl == j) {
            const double rdiag = 1.0 / rj;
#pragma unroll
            for (int i = 0; i < m; i++) t1[i] = t1[i] * rdiag;
          }
          double xj[m];
#pragma unroll
          for (int i = 0; i < m; i++) xj[i] = row_bcast<j>(t1[i]);
          if (tl > j && colx) {
#pragma unroll
            for (int i = 0; i < m; i++) t1[i] = fma(-rj, xj[i], t1[i]);
          }
          if (tl == j) {
#pragma unroll
            for (int i = 0; i < m; i++) busA[TB + j * m + i] = t1[i];
          }
          tag_store(&t1f[j]);
        });
        DPROF(14);
      } else {
        // ---------------------------------------------------------------- D: tmp2 = chol_minus(Q.uu, tmp1)
        // (backward_pass.jl:186-192, contract v4): k_bwd_team's systolic schedule, step t as row t of
        // tmp1 is released (lane 0 takes it; the rows move one lane per step)
        // lane i's row of the Q.uu factor is first used at step i (its first active step): it is loaded
        // there, as row i is released (the lanes' earlier results are never consumed)
        DPROF(17);
        double u[m], w[m], x0[m];
#pragma unroll
        for (int kk = 0; kk < m; kk++) {
          u[kk] = 0.0;
          w[kk] = 0.0;
        }
        double ru = 1.0 / u[0];
        bool okd = true;
        auto chol_step = [&](int t) {
          const int r = t - tl;
          const bool act = colu && r >= 0 && r < n;
          double x[m];
#pragma unroll
          for (int kk = 0; kk + 1 < m; kk++) x[kk] = row_shr1_or(w[kk + 1], x0[kk]);  // (lane 0: x0)
          x[m - 1] = (tl == 0) ? x0[m - 1] : 0.0;
          const double sn = x[0] * ru;
          const double s2 = sn * sn;
          okd = okd && !(act && s2 > 1.0);
          const double y = 1.0 - s2;
          const double rc = tog_rsqrt(y);
          const double cs = tog_rs_c(y, rc);
          w[0] = x[0];
#pragma unroll
          for (int kk = 1; kk < m; kk++) {
            const double tmp = (u[kk] - sn * x[kk]) * rc;
            w[kk] = cs * x[kk] - sn * tmp;
            u[kk] = act ? tmp : u[kk];
          }
          u[0] = act ? cs * u[0] : u[0];
          ru = act ? ru * rc : ru;
        };
        static_for<0, n>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          if constexpr (t < m) {
            tag_wait(&qurf[t]);
            if (tl == t) {
#pragma unroll
              for (int kk = 0; kk < m; kk++) u[kk] = (t + kk < m) ? QU[t + m * (t + kk)] : 0.0;
              ru = 1.0 / u[0];
            }
          }
          tag_wait(&t1f[t]);
#pragma unroll
          for (int kk = 0; kk < m; kk++) x0[kk] = busA[TB + t * m + kk];
          chol_step(t);
        });
        DPROF(18);
        static_for<n, n + m - 1>([&](auto tc) { chol_step(decltype(tc)::value); });  // (lane 0 idle: input row n-1)
        const unsigned long long rowmask = 0xFFFFull << (threadIdx.x & 48);
        const bool pd_fail = (__ballot(!okd) & rowmask) != 0ull;
        if (colu) {
#pragma unroll
          for (int jj = 0; jj < m; jj++)
            if (jj < tl) bus2[2 * m * m + tl + m * jj] = 0.0;
#pragma unroll
          for (int kk = 0; kk < m; kk++)
            if (tl + kk < m) bus2[2 * m * m + tl + m * (tl + kk)] = u[kk];
        }
        if (threadIdx.x == 192) flg[2] = pd_fail ? 1 : 0;
        DPROF(19);
      }
      if (faithful) kmin = k < kmin ? k : kmin;
      __syncthreads();  // B2b: tmp2, the verdict and the downdate's failure flag on the bus
      DPROF(wv == 0 ? 4 : (wv == 1 ? 10 : (wv == 2 ? 15 : 26)));
      if (flg[0] == 0) {
        // non-PD / cond > 1e8: increase ρ and restart at N-1; Q blocks are NOT re-expanded (A.1)
        if (!faithful) {
          faithful = true;  // replay this call from its start in faithful mode
          s.rho = rho0;
          s.drho = drho0;
          restarts = 0;
          kmin = N - 1;
        } else {
          reg_increase(P, s);
          restarts++;
          if (restarts > TOG_BP_MAX_RESTARTS) {
            s.flags |= TOG_TRAJ_MAX_REG | TOG_TRAJ_BP_ABORTED;
            done = true;
          }
        }
        restart = true;
        break;
      }
      if (flg[2]) {  // lowrankdowndate! throws PosDefException: this trajectory's solve stops
        s.flags |= TOG_TRAJ_SQRT_PD_FAIL | TOG_TRAJ_BP_ABORTED;
        done = true;
        restart = true;
        break;
      }
      // ------------------------------------------------------------------ S_k = qr([Q.xx + tmp1 K; tmp2 K]).R
      if (wv == 0) {
        if (k > 0) load_qxx(k - 1, Qxn);  // (in flight during the S-update)
        const double* U2p = bus2 + 2 * m * m;  // tmp2
        double a[RS];
#pragma unroll
        for (int i = 0; i < n; i++) a[i] = a2[i];
#pragma unroll
        for (int i = 0; i < m; i++) {
          double v = 0.0;
#pragma unroll
          for (int l = 0; l < m; l++) v = fma(U2p[i + m * l], Kc[l], v);
          a[n + i] = v;
        }
        // release row j of S_k after column step j: the row (zeros left of the diagonal), then its tag
        auto release = [&](auto jc, const double (&r)[RS]) {
          constexpr int j = decltype(jc)::value;
          *(colx ? Sreg + j + n * tl : pad + tl) = (j <= tl) ? r[j] : 0.0;
          tag_store(&rowf[j]);
        };
        team_qr<RS, n, 0, TEAM, false>(a, RS, tl, busA, release);
        if (store_S && colx) {
#pragma unroll
          for (int i = 0; i < n; i++) Bf.Sdbg[((size_t)b * N + k) * n * n + i + n * tl] = (i <= tl) ? a[i] : 0.0;
        }
        DPROF(5);
      } else if (wv == 2 && k > 0) {
        load_cqr(k - 1);
      } else if (wv == 1 && k > 0) {  // the next knot's S_k A_{k-1} and S_k B_{k-1}, row by row
        load_ab(k - 1, Ac, Bc);
        load_b(k - 1, Bxs, Bqu, Bquu);
        double tq[m] = {};
        static_for<0, n>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          tag_wait(&rowf[i]);
          row_products(ic, Ac, Bc, Tb, tq);
        });
        products_done(tq);
        DPROF(11);
      }
      __syncthreads();  // B3: S_k for the next knot, S_k A_{k-1} and S_k B_{k-1} on the bus
      DPROF(wv == 0 ? 25 : (wv == 1 ? 12 : (wv == 2 ? 16 : 27)));
    }
    if (!restart) done = true;
  }
  if (wv == 1) {
    const bool aborted = (s.flags & TOG_TRAJ_BP_ABORTED) != 0;
    if (!aborted) reg_decrease(P, s);  // regularization_update!(solver, :decrease) (backward_pass.jl:166)
    if (threadIdx.x == 64) {
      TrajState& g = Bf.st[b];
      g.rho = s.rho;
      g.drho = s.drho;
      g.flags = s.flags;
      g.dV0 = aborted ? 0.0 : dV0;
      g.dV1 = aborted ? 0.0 : dV1;
      g.bp_restarts = restarts + (faithful ? 1 : 0);
      if (aborted) g.active = 0;
    }
  }
  BPROF_FLUSH
}

}  // namespace tog
