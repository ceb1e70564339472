/*
 * quad_oracle.c -- TEST INFRASTRUCTURE ONLY (see quad_oracle.h for the pinning status).
 *
 * A float64 CPU restatement of the reference's hot path, used only as the checker of the
 * HIP kernels (tests/, __graft_entry__.smoke()) and as bench.py's cpu_baseline ("port").
 *
 * Part 1 restates mujoco.mj_step (third-party MuJoCo 3.x, absent here, version unpinned by the
 * reference) for model/drone/drone.xml, following MuJoCo's own pipeline and conventions:
 *   mj_step -> mj_checkPos/mj_checkVel -> mj_forward { mj_kinematics, mj_comPos, mj_crb,
 *   mj_factorM, mj_comVel, mj_passive -> mj_fluid -> mj_inertiaBoxFluidModel, mj_rne,
 *   mj_transmission (site), mj_fwdActuation, mj_fwdAcceleration } -> mj_checkAcc -> mj_Euler
 *   -> mj_advance -> mj_integratePos (mju_quatIntegrate).
 * It is deliberately the *generic* com-frame spatial-algebra formulation (cdof, cinert, CRB,
 * RNE, LTDL), so that it is an independent derivation from the structured closed form used by
 * the HIP kernel (uav_reinforcement_learning_control_amd/csrc/quad_physics.h).
 *
 * Part 2 restates the env layer: HoverEnv (envs/hover_env.py), QuadState
 * (utils/state.py), normalize/denormalize (utils/normalization.py), RateControlWrapper
 * (envs/rate_wrapper.py), TrajectoryFollowEnv's differences (envs/trajectory_follow_env.py),
 * with the reference's float32/float64 dtype flow reproduced operation by operation.
 *
 * Build: gcc -O2 -ffp-contract=off (oracle/Makefile). FMA contraction must stay off: the
 * reference's float32 normalize/denormalize are evaluated by NumPy without contraction.
 */
#include "quad_oracle.h"

#include <math.h>
#include <string.h>

#define NB 6
#define NV 10
#define MJMINVAL 1e-15
#define MJMAXVAL 1e10

/* ---------------------------------------------------------------------------------------
 * Model: model/drone/drone.xml (bodies :34-72, sites :73-76, actuators :81-84).
 * ------------------------------------------------------------------------------------- */
static const int body_parent[NB] = {-1, 0, 1, 1, 1, 1};
static const double body_pos[NB][3] = {
    {0, 0, 0},
    {0, 0, 0},                             /* base_link pos="0 0 0"          :34 */
    {0.039799, -0.039799, 0.0336},         /* prop1                          :53 */
    {-0.039799, -0.039799, 0.032484},      /* prop2                          :58 */
    {-0.039799, 0.039799, 0.033094},       /* prop3                          :63 */
    {0.039799, 0.039799, 0.0336}};         /* prop4                          :68 */
static const double body_ipos[NB][3] = {
    {0, 0, 0}, {0, 0, 0},                  /* base inertial pos="0 0 0"      :50 */
    {0, 0, -0.001}, {0, 0, 0.000116422}, {0, 0, -0.000494174}, {0, 0, -0.001}};
static const double body_iquat[NB][4] = {
    {1, 0, 0, 0}, {1, 0, 0, 0},
    {0.5, 0.5, -0.5, 0.5}, {0.5, 0.5, -0.5, 0.5}, {0.5, 0.5, -0.5, 0.5}, {0.5, 0.5, -0.5, 0.5}};
static const double body_mass[NB] = {0, 0.195, 0.00693608, 0.00693608, 0.00693608, 0.00693608};
static const double body_inertia[NB][3] = {
    {0, 0, 0},
    {4.16e-4, 4.23e-4, 5.37e-4},
    {3.75335e-06, 1.87898e-06, 1.87898e-06}, {3.75335e-06, 1.87898e-06, 1.87898e-06},
    {3.75335e-06, 1.87898e-06, 1.87898e-06}, {3.75335e-06, 1.87898e-06, 1.87898e-06}};
/* dofs: 0-5 free joint of base_link (:35), 6-9 hinge props (:55,60,65,70) */
static const int dof_body[NV] = {1, 1, 1, 1, 1, 1, 2, 3, 4, 5};
static const int dof_parent[NV] = {-1, 0, 1, 2, 3, 4, 5, 5, 5, 5};
/* actuator gear[5] (:81-84); gear[2] = 1 for all four; ctrlrange 0..13 (:9) */
static const double act_gear5[4] = {0.0201, -0.0201, 0.0201, -0.0201};
static const double ctrl_lo = 0.0, ctrl_hi = 13.0;
/* qpos0: free joint at body pos with identity quat, hinges at 0 */
static const double qpos0[ORACLE_NQ] = {0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0};

/* ---------------------------------------------------------------------------------------
 * small math (MuJoCo engine_util_* semantics)
 * ------------------------------------------------------------------------------------- */
static void quat2mat(const double q[4], double R[9]) { /* mju_quat2Mat */
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
    return;
  }
  const double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  const double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  const double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  R[0] = q00 + q11 - q22 - q33; R[4] = q00 - q11 + q22 - q33; R[8] = q00 - q11 - q22 + q33;
  R[1] = 2 * (q12 - q03); R[2] = 2 * (q13 + q02);
  R[3] = 2 * (q12 + q03); R[5] = 2 * (q23 - q01);
  R[6] = 2 * (q13 - q02); R[7] = 2 * (q23 + q01);
}
static void mulquat(double r[4], const double a[4], const double b[4]) { /* mju_mulQuat */
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof t);
}
static double normalize4(double q[4]) { /* mju_normalize4 */
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MJMINVAL) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - 1) > MJMINVAL) {
    const double inv = 1 / n;
    for (int i = 0; i < 4; i++) q[i] *= inv;
  }
  return n;
}
static double normalize3(double v[3]) { /* mju_normalize3 */
  const double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < MJMINVAL) {
    v[0] = 1; v[1] = v[2] = 0;
  } else {
    const double inv = 1 / n;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
  }
  return n;
}
static void axisangle2quat(double q[4], const double ax[3], double angle) {
  if (angle == 0) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else {
    const double s = sin(angle * 0.5);
    q[0] = cos(angle * 0.5); q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
  }
}
static void matvec3(double r[3], const double M[9], const double v[3]) {
  double t[3];
  for (int i = 0; i < 3; i++) t[i] = M[3 * i] * v[0] + M[3 * i + 1] * v[1] + M[3 * i + 2] * v[2];
  memcpy(r, t, sizeof t);
}
static void mattvec3(double r[3], const double M[9], const double v[3]) {
  double t[3];
  for (int i = 0; i < 3; i++) t[i] = M[i] * v[0] + M[3 + i] * v[1] + M[6 + i] * v[2];
  memcpy(r, t, sizeof t);
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof t);
}
static double dot(const double* a, const double* b, int n) {
  double s = 0;
  for (int i = 0; i < n; i++) s += a[i] * b[i];
  return s;
}
static int isbad(double x) { return x != x || x > MJMAXVAL || x < -MJMAXVAL; } /* mju_isBad */

/* spatial algebra, motion/force vectors as [rot(3); lin(3)] (mju_crossMotion/mju_crossForce) */
static void cross_motion(double r[6], const double v[6], const double u[6]) {
  double t[6];
  cross3(t, v, u);
  double a[3], b[3];
  cross3(a, v, u + 3);
  cross3(b, v + 3, u);
  for (int i = 0; i < 3; i++) t[3 + i] = a[i] + b[i];
  memcpy(r, t, sizeof t);
}
static void cross_force(double r[6], const double v[6], const double f[6]) {
  double a[3], b[3], c[3];
  cross3(a, v, f);         /* w x f_rot */
  cross3(b, v + 3, f + 3); /* v x f_lin */
  cross3(c, v, f + 3);     /* w x f_lin */
  for (int i = 0; i < 3; i++) { r[i] = a[i] + b[i]; r[3 + i] = c[i]; }
}
/* com-based spatial inertia as a dense 6x6 (mju_inertCom semantics) */
static void inert_com(double S[36], const double inert[3], const double mat[9], const double d[3],
                      double mass) {
  memset(S, 0, 36 * sizeof(double));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += mat[3 * i + k] * inert[k] * mat[3 * j + k];
      S[6 * i + j] = s + mass * ((i == j ? dot(d, d, 3) : 0) - d[i] * d[j]);
    }
  /* top-right m[d]x, bottom-left -m[d]x, bottom-right m*I */
  const double dx[9] = {0, -d[2], d[1], d[2], 0, -d[0], -d[1], d[0], 0};
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      S[6 * i + 3 + j] = mass * dx[3 * i + j];
      S[6 * (3 + i) + j] = -mass * dx[3 * i + j];
      S[6 * (3 + i) + 3 + j] = (i == j) ? mass : 0;
    }
}
static void mul6(double r[6], const double S[36], const double v[6]) {
  double t[6];
  for (int i = 0; i < 6; i++) t[i] = dot(S + 6 * i, v, 6);
  memcpy(r, t, sizeof t);
}

/* ---------------------------------------------------------------------------------------
 * mj_forward pieces
 * ------------------------------------------------------------------------------------- */
typedef struct Kin {
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], ximat[NB][9];
  double xanchor[NB][3], xaxis[NB][3];
  double com[3];                 /* subtree_com of the root body (body_rootid = 1 for 1..5) */
  double cinert[NB][36];
  double cdof[NV][6], cdofdot[NV][6];
  double cvel[NB][6];
} Kin;

static void mj_kinematics(const double* qpos, Kin* k) {
  memset(k, 0, sizeof *k);
  k->xquat[0][0] = 1;
  quat2mat(k->xquat[0], k->xmat[0]);
  quat2mat(k->xquat[0], k->ximat[0]);
  /* free joint body: copy pos and normalized quat from qpos */
  for (int i = 0; i < 3; i++) k->xpos[1][i] = qpos[i];
  for (int i = 0; i < 4; i++) k->xquat[1][i] = qpos[3 + i];
  normalize4(k->xquat[1]);
  memcpy(k->xanchor[1], k->xpos[1], sizeof k->xpos[1]);
  k->xaxis[1][2] = 1;
  quat2mat(k->xquat[1], k->xmat[1]);
  /* hinge bodies: fixed offset in the parent, then rotation about local z by qpos[7+i] */
  for (int b = 2; b < NB; b++) {
    const int p = body_parent[b];
    matvec3(k->xpos[b], k->xmat[p], body_pos[b]);
    for (int i = 0; i < 3; i++) k->xpos[b][i] += k->xpos[p][i];
    memcpy(k->xquat[b], k->xquat[p], sizeof k->xquat[p]); /* body quat = identity */
    double R[9];
    quat2mat(k->xquat[b], R);
    const double zax[3] = {0, 0, 1};
    matvec3(k->xaxis[b], R, zax);
    memcpy(k->xanchor[b], k->xpos[b], sizeof k->xpos[b]); /* jnt_pos = 0 */
    double qloc[4];
    axisangle2quat(qloc, zax, qpos[7 + (b - 2)] - qpos0[7 + (b - 2)]);
    mulquat(k->xquat[b], k->xquat[b], qloc);
    normalize4(k->xquat[b]);
    quat2mat(k->xquat[b], k->xmat[b]);
  }
  /* mj_local2Global for the inertial frames */
  for (int b = 1; b < NB; b++) {
    matvec3(k->xipos[b], k->xmat[b], body_ipos[b]);
    for (int i = 0; i < 3; i++) k->xipos[b][i] += k->xpos[b][i];
    double q[4];
    mulquat(q, k->xquat[b], body_iquat[b]);
    quat2mat(q, k->ximat[b]);
  }
}

static void mj_comPos(Kin* k) {
  double msum = 0;
  for (int b = 1; b < NB; b++) {
    for (int i = 0; i < 3; i++) k->com[i] += body_mass[b] * k->xipos[b][i];
    msum += body_mass[b];
  }
  for (int i = 0; i < 3; i++) k->com[i] /= msum;
  for (int b = 1; b < NB; b++) {
    double d[3];
    for (int i = 0; i < 3; i++) d[i] = k->xipos[b][i] - k->com[i];
    inert_com(k->cinert[b], body_inertia[b], k->ximat[b], d, body_mass[b]);
  }
  /* cdof: free translation along world axes, free rotation about body axes through the
   * anchor, hinge rotation about xaxis through its anchor (mju_dofCom). */
  memset(k->cdof, 0, sizeof k->cdof);
  for (int j = 0; j < 3; j++) k->cdof[j][3 + j] = 1;
  double off[3];
  for (int i = 0; i < 3; i++) off[i] = k->com[i] - k->xanchor[1][i];
  for (int j = 0; j < 3; j++) {
    const double ax[3] = {k->xmat[1][j], k->xmat[1][3 + j], k->xmat[1][6 + j]};
    memcpy(k->cdof[3 + j], ax, sizeof ax);
    cross3(k->cdof[3 + j] + 3, ax, off);
  }
  for (int b = 2; b < NB; b++) {
    const int j = 6 + (b - 2);
    for (int i = 0; i < 3; i++) off[i] = k->com[i] - k->xanchor[b][i];
    memcpy(k->cdof[j], k->xaxis[b], 3 * sizeof(double));
    cross3(k->cdof[j] + 3, k->xaxis[b], off);
  }
}

static void mj_crb(const Kin* k, double M[NV][NV]) {
  double crb[NB][36];
  memcpy(crb, k->cinert, sizeof crb);
  for (int b = NB - 1; b > 1; b--)
    for (int i = 0; i < 36; i++) crb[body_parent[b]][i] += crb[b][i];
  memset(M, 0, sizeof(double) * NV * NV);
  for (int i = 0; i < NV; i++) {
    double buf[6];
    mul6(buf, crb[dof_body[i]], k->cdof[i]);
    for (int j = i; j >= 0; j = dof_parent[j]) {
      M[i][j] = dot(k->cdof[j], buf, 6);
      M[j][i] = M[i][j];
    }
  }
}

static void mj_comVel(Kin* k, const double* qvel) {
  memset(k->cvel, 0, sizeof k->cvel);
  memset(k->cdofdot, 0, sizeof k->cdofdot);
  /* free joint: translation dofs have cdofdot = 0, rotation dofs use the velocity after the
   * translation part has been added; hinge dofs use the parent velocity. */
  double cvel[6] = {0};
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 6; i++) cvel[i] += k->cdof[j][i] * qvel[j];
  for (int j = 3; j < 6; j++) cross_motion(k->cdofdot[j], cvel, k->cdof[j]);
  for (int j = 3; j < 6; j++)
    for (int i = 0; i < 6; i++) cvel[i] += k->cdof[j][i] * qvel[j];
  memcpy(k->cvel[1], cvel, sizeof cvel);
  for (int b = 2; b < NB; b++) {
    const int j = 6 + (b - 2);
    cross_motion(k->cdofdot[j], k->cvel[1], k->cdof[j]);
    for (int i = 0; i < 6; i++) k->cvel[b][i] = k->cvel[1][i] + k->cdof[j][i] * qvel[j];
  }
}

/* mj_applyFT: qfrc += J_p(point, body)' f + J_r(body)' t */
static void apply_ft(const Kin* k, const double f[3], const double t[3], const double pt[3],
                     int body, double* qfrc) {
  double off[3];
  for (int i = 0; i < 3; i++) off[i] = pt[i] - k->com[i];
  for (int j = 0; j < NV; j++) {
    /* dof j affects body iff dof_body[j] is body or an ancestor of it */
    int b = body, on = 0;
    while (b > 0) { if (b == dof_body[j]) { on = 1; break; } b = body_parent[b]; }
    if (!on) continue;
    double jp[3];
    cross3(jp, k->cdof[j], off);
    for (int i = 0; i < 3; i++) jp[i] += k->cdof[j][3 + i];
    qfrc[j] += dot(jp, f, 3) + dot(k->cdof[j], t, 3);
  }
}

/* mj_inertiaBoxFluidModel for body b */
static void fluid_box(const OracleOpt* opt, const Kin* k, int b, double* qfrc) {
  const double* in = body_inertia[b];
  const double m = body_mass[b];
  double box[3];
  box[0] = sqrt(fmax(MJMINVAL, in[1] + in[2] - in[0]) / m * 6.0);
  box[1] = sqrt(fmax(MJMINVAL, in[0] + in[2] - in[1]) / m * 6.0);
  box[2] = sqrt(fmax(MJMINVAL, in[0] + in[1] - in[2]) / m * 6.0);
  /* mj_objectVelocity(flg_local=1): velocity at xipos in the ximat frame */
  double dif[3], cr[3], tran[6], lvel[6];
  for (int i = 0; i < 3; i++) dif[i] = k->xipos[b][i] - k->com[i];
  cross3(cr, dif, k->cvel[b]);
  for (int i = 0; i < 3; i++) { tran[i] = k->cvel[b][i]; tran[3 + i] = k->cvel[b][3 + i] - cr[i]; }
  mattvec3(lvel, k->ximat[b], tran);
  mattvec3(lvel + 3, k->ximat[b], tran + 3);
  /* wind = 0 */
  double lfrc[6] = {0};
  if (opt->viscosity > 0) {
    const double diam = (box[0] + box[1] + box[2]) / 3.0;
    for (int i = 0; i < 3; i++) lfrc[i] = -M_PI * diam * diam * diam * opt->viscosity * lvel[i];
    for (int i = 0; i < 3; i++) lfrc[3 + i] = -3.0 * M_PI * diam * opt->viscosity * lvel[3 + i];
  }
  if (opt->density > 0) {
    const double rho = opt->density;
    lfrc[3] -= 0.5 * rho * box[1] * box[2] * fabs(lvel[3]) * lvel[3];
    lfrc[4] -= 0.5 * rho * box[0] * box[2] * fabs(lvel[4]) * lvel[4];
    lfrc[5] -= 0.5 * rho * box[0] * box[1] * fabs(lvel[5]) * lvel[5];
    const double b4[3] = {pow(box[0], 4), pow(box[1], 4), pow(box[2], 4)};
    lfrc[0] -= rho * box[0] * (b4[1] + b4[2]) * fabs(lvel[0]) * lvel[0] / 64.0;
    lfrc[1] -= rho * box[1] * (b4[0] + b4[2]) * fabs(lvel[1]) * lvel[1] / 64.0;
    lfrc[2] -= rho * box[2] * (b4[0] + b4[1]) * fabs(lvel[2]) * lvel[2] / 64.0;
  }
  double bfrc[6];
  matvec3(bfrc, k->ximat[b], lfrc);
  matvec3(bfrc + 3, k->ximat[b], lfrc + 3);
  apply_ft(k, bfrc + 3, bfrc, k->xipos[b], b, qfrc);
}

/* mj_rne with flg_acc = 0 */
static void mj_rne(const OracleOpt* opt, const Kin* k, const double* qvel, double* bias) {
  double cacc[NB][6], cfrc[NB][6];
  memset(cacc, 0, sizeof cacc);
  memset(cfrc, 0, sizeof cfrc);
  for (int i = 0; i < 3; i++) cacc[0][3 + i] = -opt->gravity[i];
  for (int b = 1; b < NB; b++) {
    const int p = body_parent[b];
    for (int i = 0; i < 6; i++) cacc[b][i] = cacc[p][i];
    for (int j = 0; j < NV; j++)
      if (dof_body[j] == b)
        for (int i = 0; i < 6; i++) cacc[b][i] += k->cdofdot[j][i] * qvel[j];
    double t1[6], t2[6];
    mul6(cfrc[b], k->cinert[b], cacc[b]);
    mul6(t1, k->cinert[b], k->cvel[b]);
    cross_force(t2, k->cvel[b], t1);
    for (int i = 0; i < 6; i++) cfrc[b][i] += t2[i];
  }
  for (int b = NB - 1; b > 0; b--)
    if (body_parent[b] > 0)
      for (int i = 0; i < 6; i++) cfrc[body_parent[b]][i] += cfrc[b][i];
  for (int j = 0; j < NV; j++) bias[j] = dot(k->cdof[j], cfrc[dof_body[j]], 6);
}

/* mj_transmission (site, no refsite) + mj_fwdActuation (motor: gain 1, no bias) */
static void mj_actuation(const Kin* k, const double* ctrl, double* qfrc) {
  memset(qfrc, 0, NV * sizeof(double));
  for (int a = 0; a < 4; a++) {
    double spos[3];
    matvec3(spos, k->xmat[1], body_pos[2 + a]); /* site_pos == prop body pos; site on base */
    for (int i = 0; i < 3; i++) spos[i] += k->xpos[1][i];
    const double gear_f[3] = {0, 0, 1}, gear_t[3] = {0, 0, act_gear5[a]};
    double wf[3], wt[3];
    matvec3(wf, k->xmat[1], gear_f);
    matvec3(wt, k->xmat[1], gear_t);
    double f[3], t[3];
    for (int i = 0; i < 3; i++) { f[i] = wf[i] * ctrl[a]; t[i] = wt[i] * ctrl[a]; }
    apply_ft(k, f, t, spos, 1, qfrc);
  }
}

/* mj_factorM + mj_solveM: reverse-order L'DL of the tree-structured mass matrix */
static void solve_m(const double Min[NV][NV], const double* b, double* x) {
  double L[NV][NV];
  memcpy(L, Min, sizeof L);
  for (int k = NV - 1; k >= 0; k--) {
    if (L[k][k] < MJMINVAL) L[k][k] = MJMINVAL;
    for (int i = dof_parent[k]; i >= 0; i = dof_parent[i]) {
      const double tmp = L[k][i] / L[k][k];
      for (int j = i; j >= 0; j = dof_parent[j]) L[i][j] -= tmp * L[k][j];
      L[k][i] = tmp;
    }
  }
  for (int i = 0; i < NV; i++) x[i] = b[i];
  for (int k = NV - 1; k >= 0; k--)
    for (int i = dof_parent[k]; i >= 0; i = dof_parent[i]) x[i] -= L[k][i] * x[k];
  for (int k = 0; k < NV; k++) x[k] /= L[k][k];
  for (int k = 0; k < NV; k++)
    for (int i = dof_parent[k]; i >= 0; i = dof_parent[i]) x[k] -= L[k][i] * x[i];
}

static void forward_full(const OracleOpt* opt, const double* qpos, const double* qvel,
                         const double* ctrl, double M[NV][NV], double* bias, double* passive,
                         double* actf, double* qacc) {
  Kin k;
  mj_kinematics(qpos, &k);
  mj_comPos(&k);
  mj_crb(&k, M);
  mj_comVel(&k, qvel);
  memset(passive, 0, NV * sizeof(double));
  if (opt->viscosity > 0 || opt->density > 0)
    for (int b = 1; b < NB; b++) fluid_box(opt, &k, b, passive);
  mj_rne(opt, &k, qvel, bias);
  mj_actuation(&k, ctrl, actf);
  double f[NV];
  for (int i = 0; i < NV; i++) f[i] = passive[i] + actf[i] - bias[i];
  solve_m((const double(*)[NV])M, f, qacc);
}

void oracle_mj_forward(const OracleOpt* opt, const double* qpos, const double* qvel,
                       const double* ctrl, double* Mout, double* bias, double* passive,
                       double* actf, double* qacc) {
  double M[NV][NV], b[NV], p[NV], a[NV], q[NV], c[4];
  for (int i = 0; i < 4; i++) {
    c[i] = ctrl[i];
    if (c[i] < ctrl_lo) c[i] = ctrl_lo; else if (c[i] > ctrl_hi) c[i] = ctrl_hi;
  }
  forward_full(opt, qpos, qvel, c, M, b, p, a, q);
  if (Mout) memcpy(Mout, M, sizeof M);
  if (bias) memcpy(bias, b, sizeof b);
  if (passive) memcpy(passive, p, sizeof p);
  if (actf) memcpy(actf, a, sizeof a);
  if (qacc) memcpy(qacc, q, sizeof q);
}

static void reset_data(double* qpos, double* qvel, double* ctrl) { /* mj_resetData */
  memcpy(qpos, qpos0, sizeof qpos0);
  memset(qvel, 0, NV * sizeof(double));
  memset(ctrl, 0, 4 * sizeof(double));
}

/* mj_Euler (no dof damping) -> mj_advance: semi-implicit Euler */
static void euler_advance(const OracleOpt* opt, double* qpos, double* qvel, const double* qacc) {
  const double h = opt->timestep;
  for (int i = 0; i < NV; i++) qvel[i] += h * qacc[i];
  for (int i = 0; i < 3; i++) qpos[i] += h * qvel[i];
  { /* mju_quatIntegrate(qpos+3, qvel+3, h) */
    double ax[3] = {qvel[3], qvel[4], qvel[5]}, qrot[4];
    const double angle = h * normalize3(ax);
    axisangle2quat(qrot, ax, angle);
    normalize4(qpos + 3);
    mulquat(qpos + 3, qpos + 3, qrot);
  }
  for (int i = 0; i < 4; i++) qpos[7 + i] += h * qvel[6 + i];
}

int oracle_mj_step(const OracleOpt* opt, double* qpos, double* qvel, double* ctrl) {
  int warn = 0;
  for (int i = 0; i < ORACLE_NQ; i++)
    if (isbad(qpos[i])) { reset_data(qpos, qvel, ctrl); warn |= 1; break; } /* mj_checkPos */
  for (int i = 0; i < NV; i++)
    if (isbad(qvel[i])) { reset_data(qpos, qvel, ctrl); warn |= 2; break; } /* mj_checkVel */
  /* mj_fwdActuation: bad ctrl => all ctrl zeroed (mjWARN_BADCTRL), then ctrlrange clamp */
  for (int i = 0; i < 4; i++)
    if (isbad(ctrl[i])) { memset(ctrl, 0, 4 * sizeof(double)); warn |= 4; break; }
  double c[4];
  for (int i = 0; i < 4; i++) {
    c[i] = ctrl[i];
    if (c[i] < ctrl_lo) c[i] = ctrl_lo; else if (c[i] > ctrl_hi) c[i] = ctrl_hi;
  }
  double M[NV][NV], bias[NV], passive[NV], actf[NV], qacc[NV];
  forward_full(opt, qpos, qvel, c, M, bias, passive, actf, qacc);
  for (int i = 0; i < NV; i++)
    if (isbad(qacc[i])) { /* mj_checkAcc: reset and recompute at qpos0 with ctrl = 0 */
      reset_data(qpos, qvel, ctrl);
      memset(c, 0, sizeof c);
      forward_full(opt, qpos, qvel, c, M, bias, passive, actf, qacc);
      warn |= 8;
      break;
    }
  euler_advance(opt, qpos, qvel, qacc);
  return warn;
}

/* mjx.step: the same forward dynamics and Euler step without MuJoCo C's bad-state checks
 * (MJX raises no warnings: a NaN/huge state or ctrl propagates; jnp.clip keeps NaN). */
void oracle_mjx_step(const OracleOpt* opt, double* qpos, double* qvel, const double* ctrl) {
  double c[4];
  for (int i = 0; i < 4; i++) {
    c[i] = ctrl[i];
    if (c[i] < ctrl_lo) c[i] = ctrl_lo; else if (c[i] > ctrl_hi) c[i] = ctrl_hi;
  }
  double M[NV][NV], bias[NV], passive[NV], actf[NV], qacc[NV];
  forward_full(opt, qpos, qvel, c, M, bias, passive, actf, qacc);
  euler_advance(opt, qpos, qvel, qacc);
}

/* ---------------------------------------------------------------------------------------
 * scipy.spatial.transform.Rotation restatements (scipy 1.15, used by utils/state.py)
 * ------------------------------------------------------------------------------------- */
void oracle_quat_to_euler(const double q_wxyz[4], double e[3]) {
  /* from_quat normalizes; as_euler('xyz') uses the Bernardes & Viollet (2022) algorithm:
   * extrinsic x-y-z: i=0,j=1,k=2, Tait-Bryan, sign=+1 */
  double qx = q_wxyz[1], qy = q_wxyz[2], qz = q_wxyz[3], qw = q_wxyz[0];
  const double n = sqrt(qx * qx + qy * qy + qz * qz + qw * qw);
  qx /= n; qy /= n; qz /= n; qw /= n;
  const double a = qw - qy, b = qx + qz, c = qy + qw, d = qz - qx;
  e[1] = 2 * atan2(hypot(c, d), hypot(a, b));
  const int case1 = fabs(e[1]) <= 1e-7, case2 = fabs(e[1] - M_PI) <= 1e-7;
  const double half_sum = atan2(b, a), half_diff = atan2(d, c);
  if (!(case1 || case2)) {
    e[0] = half_sum - half_diff;
    e[2] = half_sum + half_diff;
  } else {
    e[2] = 0;
    e[0] = case1 ? 2 * half_sum : -2 * half_diff;
  }
  e[1] -= M_PI / 2;
  for (int i = 0; i < 3; i++) {
    if (e[i] < -M_PI) e[i] += 2 * M_PI;
    else if (e[i] > M_PI) e[i] -= 2 * M_PI;
  }
}

/* oracle_quat_to_euler over n quaternions (wxyz rows): the tests' Euler angles of the kernel's own
 * post-step quaternions (tests/test_gpu_parity.py euler_of_quat) */
void oracle_quat_to_euler_batch(const double* q_wxyz, int32_t n, double* e) {
  for (int32_t i = 0; i < n; i++) oracle_quat_to_euler(q_wxyz + 4 * (size_t)i, e + 3 * (size_t)i);
}

void oracle_euler_to_quat(const double e[3], double q_wxyz[4]) {
  /* from_euler('xyz'): extrinsic composition q = qz * (qy * qx), elements xyzw */
  double res[4] = {sin(e[0] / 2), 0, 0, cos(e[0] / 2)};
  for (int ax = 1; ax < 3; ax++) {
    double p[4] = {0, 0, 0, cos(e[ax] / 2)};
    p[ax] = sin(e[ax] / 2);
    double cr[3], r[4];
    cross3(cr, p, res);
    for (int i = 0; i < 3; i++) r[i] = p[3] * res[i] + res[3] * p[i] + cr[i];
    r[3] = p[3] * res[3] - (p[0] * res[0] + p[1] * res[1] + p[2] * res[2]);
    memcpy(res, r, sizeof r);
  }
  q_wxyz[0] = res[3]; q_wxyz[1] = res[0]; q_wxyz[2] = res[1]; q_wxyz[3] = res[2];
}

/* ---------------------------------------------------------------------------------------
 * env layer
 * ------------------------------------------------------------------------------------- */
static double clipd(double x, double lo, double hi) { /* np.clip propagates NaN */
  if (x != x) return x;
  return x < lo ? lo : (x > hi ? hi : x);
}

void oracle_default_cfg(int32_t env_kind, int32_t wrapper, OracleCfg* c) {
  memset(c, 0, sizeof *c);
  c->env_kind = env_kind;
  c->wrapper = wrapper;
  const double pi = M_PI;
  /* hover_env.py:36-39 (identical in trajectory_follow_env.py:44-47) */
  const double ol[12] = {-4, -4, -2, -pi, -pi, -pi, -10, -10, -10, -6 * pi, -6 * pi, -6 * pi};
  /* hover_env.py:42-45, trajectory_follow_env.py:49-52 */
  const double il[12] = {-1.5, -1.5, 0.1, -0.3, -0.3, -0.3, -0.5, -0.5, -0.5, -0.5, -0.5, -0.5};
  const double ih[12] = {1.5, 1.5, 1.5, 0.3, 0.3, 0.3, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5};
  for (int i = 0; i < 12; i++) {
    c->obs_low[i] = (float)ol[i];
    c->obs_high[i] = (float)(-ol[i]);
    c->init_low[i] = (float)il[i];
    c->init_high[i] = (float)ih[i];
    c->term_low[i] = (float)ol[i];
    c->term_high[i] = (float)(-ol[i]);
  }
  if (env_kind == ORACLE_ENV_TRAJ) {
    /* trajectory_follow_env.py:60-63 */
    c->term_low[0] = -3; c->term_low[1] = -3; c->term_low[2] = 0;
    c->term_high[0] = 3; c->term_high[1] = 3; c->term_high[2] = 3;
    c->max_episode_steps = 2048;                       /* :24 */
    c->nominal_voltage = 16.8; c->min_voltage = 13.2;  /* :26 */
    /* the target is the start position (:236,242-243); the target bounds are unused */
  } else {
    /* hover_env.py:54-57 */
    c->term_low[0] = -2; c->term_low[1] = -2; c->term_low[2] = 0;
    c->term_high[0] = 2; c->term_high[1] = 2; c->term_high[2] = 2;
    c->max_episode_steps = 512;                        /* :16 */
    c->nominal_voltage = 8.4; c->min_voltage = 7.6;    /* :18 */
  }
  const float tl[3] = {-1.5f, -1.5f, 0.3f}, th[3] = {1.5f, 1.5f, 1.8f}; /* hover_env.py:48-51 */
  for (int i = 0; i < 3; i++) { c->target_low[i] = tl[i]; c->target_high[i] = th[i]; }
  c->max_motor_thrust = 13.0;       /* drone_config.py:9 */
  c->arm_length = 0.039799;         /* :10 */
  c->yaw_coeff = 0.0201;            /* :11 */
  c->max_torque = 0.5;              /* :21 */
  const double mt = 4 * c->max_motor_thrust;
  const double al[4] = {0.0, -0.5, -0.5, -0.5}, ah[4] = {mt, 0.5, 0.5, 0.5}; /* :60-65 */
  for (int i = 0; i < 4; i++) { c->act_low[i] = (float)al[i]; c->act_high[i] = (float)ah[i]; }
  c->vdrop_base = 0.01; c->vdrop_load = 0.08;
  /* rate_wrapper.py:52-58 with pid_gains.json:43-52 */
  c->rate_max_rad = 360.0 * (M_PI / 180.0);
  c->rate_kd[0] = 26; c->rate_kd[1] = 26; c->rate_kd[2] = 18;
  c->rate_ki = 0.025; c->rate_imax = 0.01;
  c->inertia[0] = 4.16e-4; c->inertia[1] = 4.23e-4; c->inertia[2] = 5.37e-4;
  c->opt.timestep = 0.01;
  c->opt.gravity[2] = -9.81;
  c->opt.density = 1.225;
  c->opt.viscosity = 1.8e-5;
}

/* np.linalg.inv(A) of the mixer (hover_env.py:94-100), Gauss-Jordan with partial pivoting */
static void mixer_inverse(const OracleCfg* c, double Ai[4][4]) {
  const double l = c->arm_length, k = c->yaw_coeff;
  double A[4][8] = {{1, 1, 1, 1}, {-l, -l, l, l}, {-l, l, l, -l}, {k, -k, k, -k}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) A[i][4 + j] = (i == j);
  for (int col = 0; col < 4; col++) {
    int piv = col;
    for (int r = col + 1; r < 4; r++) if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
    for (int j = 0; j < 8; j++) { double t = A[col][j]; A[col][j] = A[piv][j]; A[piv][j] = t; }
    const double d = A[col][col];
    for (int j = 0; j < 8; j++) A[col][j] /= d;
    for (int r = 0; r < 4; r++)
      if (r != col) {
        const double f = A[r][col];
        for (int j = 0; j < 8; j++) A[r][j] -= f * A[col][j];
      }
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) Ai[i][j] = A[i][4 + j];
}

void oracle_get_obs(const OracleCfg* cfg, OracleEnv* env, float obs[12]) {
  double eul[3];
  oracle_quat_to_euler(env->qpos + 3, eul);
  for (int i = 0; i < 3; i++) {
    env->state12[i] = (float)env->qpos[i];
    env->state12[3 + i] = (float)eul[i];
    env->state12[6 + i] = (float)env->qvel[i];
    env->state12[9 + i] = (float)env->qvel[3 + i];
  }
  float o[12];
  memcpy(o, env->state12, sizeof o);
  for (int i = 0; i < 3; i++) o[i] = env->target[i] - env->state12[i];
  for (int i = 0; i < 12; i++) {
    const float t = o[i] - cfg->obs_low[i];
    const float u = 2.0f * t;
    const float w = cfg->obs_high[i] - cfg->obs_low[i];
    const float v = u / w;
    obs[i] = v - 1.0f;
  }
}

void oracle_env_reset(const OracleCfg* cfg, OracleEnv* env, const float init12[12],
                      const float target3[3], float obs[12]) {
  double ctrl[4];
  reset_data(env->qpos, env->qvel, ctrl); /* mj_resetData (hover_env.py:216) */
  env->step_count = 0;
  env->voltage = cfg->nominal_voltage;
  for (int i = 0; i < 3; i++) env->rate_int[i] = 0.0; /* rate_wrapper.py:110 */
  for (int i = 0; i < 4; i++) env->prev_action[i] = 0.0f; /* hover_env.py:212 */
  /* QuadState.get_mujoco_state (state.py:48-65) + HoverEnv.set_state (hover_env.py:143-148) */
  const double e[3] = {init12[3], init12[4], init12[5]};
  for (int i = 0; i < 3; i++) env->qpos[i] = init12[i];
  oracle_euler_to_quat(e, env->qpos + 3);
  for (int i = 0; i < 6; i++) env->qvel[i] = init12[6 + i];
  if (cfg->env_kind == ORACLE_ENV_TRAJ) {
    for (int i = 0; i < 3; i++) env->target[i] = init12[i]; /* traj_pos[0] == start */
  } else {
    for (int i = 0; i < 3; i++) env->target[i] = target3[i];
  }
  oracle_get_obs(cfg, env, obs);
}

int oracle_env_step(const OracleCfg* cfg, OracleEnv* env, const float action[4],
                    OracleStepOut* out) {
  float a[4];
  a[0] = action[0];
  const int ctbr = cfg->wrapper == ORACLE_WRAP_CTBR || cfg->wrapper == ORACLE_WRAP_CTBR_RELPOS;
  if (ctbr) { /* RateControlWrapper.action (rate_wrapper.py:69-98) */
    const double dt = cfg->opt.timestep;
    for (int k = 0; k < 3; k++) {
      const double des = (double)action[1 + k] * cfg->rate_max_rad;
      const double err = des - (double)env->state12[9 + k];
      const double tau_p = (cfg->inertia[k] * cfg->rate_kd[k]) * err;
      env->rate_int[k] = env->rate_int[k] + (cfg->rate_ki * dt) * err;
      env->rate_int[k] = clipd(env->rate_int[k], -cfg->rate_imax, cfg->rate_imax);
      const double tau = tau_p + env->rate_int[k];
      a[1 + k] = (float)clipd(tau / cfg->max_torque, -1.0, 1.0);
    }
  } else {
    for (int k = 1; k < 4; k++) a[k] = action[k];
  }
  memcpy(out->env_action, a, sizeof a);
  /* self._prev_action = np.array(action, dtype=np.float32) (hover_env.py:166): the action the
   * base env receives; RateControlWrapper.step then overwrites it with the rate action it was
   * given (rate_wrapper.py:100-106), which is what RelPosActWrapper above it reads */
  memcpy(env->prev_action, ctbr ? action : a, sizeof a);
  /* denormalize (normalization.py:20-30), float32 */
  float phys[4];
  for (int k = 0; k < 4; k++) {
    const float s = a[k] + 1.0f;
    const float h = s / 2.0f;
    const float w = cfg->act_high[k] - cfg->act_low[k];
    const float m = h * w;
    phys[k] = m + cfg->act_low[k];
  }
  /* _mix_to_motors (hover_env.py:111-124), float64 */
  double Ai[4][4], F[4];
  mixer_inverse(cfg, Ai);
  for (int i = 0; i < 4; i++) {
    double s = 0;
    for (int j = 0; j < 4; j++) s += Ai[i][j] * (double)phys[j];
    F[i] = clipd(s, 0.0, cfg->max_motor_thrust);
  }
  /* voltage sag (hover_env.py:102-109,174-176) */
  const double vs = clipd(env->voltage / cfg->nominal_voltage, 0.0, 1.0);
  for (int i = 0; i < 4; i++) F[i] = clipd(F[i] * vs, 0.0, cfg->max_motor_thrust * vs);
  const double mean = (F[0] + F[1] + F[2] + F[3]) / 4.0;
  const double load = mean / fmax(cfg->max_motor_thrust, 1e-6);
  const double dV = (cfg->vdrop_base + cfg->vdrop_load * load) * cfg->opt.timestep;
  env->voltage = clipd(env->voltage - dV, cfg->min_voltage, cfg->nominal_voltage);
  /* data.ctrl[:] = F ; mujoco.mj_step (hover_env.py:177-180) */
  double ctrl[4];
  memcpy(ctrl, F, sizeof ctrl);
  oracle_mj_step(&cfg->opt, env->qpos, env->qvel, ctrl);
  env->step_count += 1;
  oracle_get_obs(cfg, env, out->obs);
  /* _get_reward (hover_env.py:138-141): np.linalg.norm of a float32 vector is sqrt(x.dot(x)),
   * and NumPy's BLAS sdot rounds each product to float32 and accumulates in float64 (matched
   * bit-exactly against the golden vectors); then float64 exp. */
  float d[3];
  double acc = 0.0;
  for (int i = 0; i < 3; i++) d[i] = env->state12[i] - env->target[i];
  for (int i = 0; i < 3; i++) { const float p = d[i] * d[i]; acc += (double)p; }
  const double pe = (double)sqrtf((float)acc);
  out->reward = exp(-(pe * pe));
  /* _is_terminated (hover_env.py:150-157) + truncation (:188) */
  int term = 0;
  for (int i = 0; i < 12; i++) {
    const float s = env->state12[i];
    if (!isfinite(s)) term = 1;
    if (!(s >= cfg->term_low[i] && s <= cfg->term_high[i])) term = 1;
  }
  out->terminated = term;
  out->truncated = env->step_count >= cfg->max_episode_steps;
  memcpy(out->state12, env->state12, sizeof out->state12);
  memcpy(out->motor_commands, F, sizeof F);
  out->voltage = env->voltage;
  out->voltage_scale = vs;
  oracle_relpos_obs(env, out->obs, out->obs7);
  return 0;
}

void oracle_relpos_obs(const OracleEnv* env, const float obs12[12], float obs7[7]) {
  /* np.concatenate([obs[0:3], self.unwrapped._prev_action]).astype(np.float32) */
  for (int i = 0; i < 3; i++) obs7[i] = obs12[i];
  for (int i = 0; i < 4; i++) obs7[3 + i] = env->prev_action[i];
}

void oracle_env_step_batch(const OracleCfg* cfg, OracleEnv* envs, int32_t n,
                           const float* actions, OracleStepOut* outs) {
  for (int32_t i = 0; i < n; i++) oracle_env_step(cfg, envs + i, actions + 4 * i, outs + i);
}

/* Batch helpers for the large-N parity tests (test infrastructure only): derive every env's
 * state12 from its (qpos, qvel) as set_full_state does, and reset a batch from given draws. */
void oracle_env_prepare_batch(const OracleCfg* cfg, OracleEnv* envs, int32_t n) {
  float obs[12];
  for (int32_t i = 0; i < n; i++) oracle_get_obs(cfg, envs + i, obs);
}

void oracle_env_reset_batch(const OracleCfg* cfg, OracleEnv* envs, int32_t n, const float* init12,
                            const float* target3, float* obs) {
  for (int32_t i = 0; i < n; i++)
    oracle_env_reset(cfg, envs + i, init12 + 12 * (size_t)i, target3 + 3 * (size_t)i, obs + 12 * (size_t)i);
}

/* ---------------------------------------------------------------------------------------
 * Philox4x32-10 and the device draw mapping (restated for reset/action parity)
 * ------------------------------------------------------------------------------------- */
void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr_in[0], ctr_in[1], ctr_in[2], ctr_in[3]};
  uint32_t k[2] = {key_in[0], key_in[1]};
  for (int r = 0; r < 10; r++) {
    if (r > 0) { k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
  }
  memcpy(out, c, sizeof c);
}

static float u01(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

void oracle_reset_draw(const OracleCfg* cfg, uint64_t seed, uint64_t gid, uint32_t episode,
                       float init12[12], float target3[3]) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t r[16];
  for (uint32_t blk = 0; blk < 4; blk++) {
    const uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), episode, blk};
    oracle_philox4x32_10(ctr, key, r + 4 * blk);
  }
  for (int i = 0; i < 12; i++) {
    const float w = cfg->init_high[i] - cfg->init_low[i];
    const float m = u01(r[i]) * w;
    init12[i] = cfg->init_low[i] + m;
  }
  for (int i = 0; i < 3; i++) {
    const float w = cfg->target_high[i] - cfg->target_low[i];
    const float m = u01(r[12 + i]) * w;
    target3[i] = cfg->target_low[i] + m;
  }
}

void oracle_reset_draw_batch(const OracleCfg* cfg, uint64_t seed, const uint64_t* gid,
                             const uint32_t* episode, int32_t n, float* init12, float* target3) {
  for (int32_t i = 0; i < n; i++)
    oracle_reset_draw(cfg, seed, gid[i], episode[i], init12 + 12 * (size_t)i, target3 + 3 * (size_t)i);
}

void oracle_random_action(uint64_t seed, uint64_t gid, uint32_t step, float a[4]) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), step, 0x100u};
  uint32_t r[4];
  oracle_philox4x32_10(ctr, key, r);
  for (int i = 0; i < 4; i++) a[i] = (float)(r[i] >> 8) * 0x1p-23f - 1.0f;
}

double oracle_bench_rollout(const OracleCfg* cfg, int32_t n_envs, int32_t n_steps, uint64_t seed) {
  OracleEnv envs[64];
  uint32_t ep[64];
  if (n_envs > 64) n_envs = 64;
  double sum = 0;
  float obs[12], i12[12], t3[3], a[4];
  for (int i = 0; i < n_envs; i++) {
    oracle_reset_draw(cfg, seed, (uint64_t)i, 0, i12, t3);
    oracle_env_reset(cfg, &envs[i], i12, t3, obs);
    ep[i] = 1;
  }
  OracleStepOut out;
  for (int t = 0; t < n_steps; t++)
    for (int i = 0; i < n_envs; i++) {
      oracle_random_action(seed, (uint64_t)i, (uint32_t)t, a);
      oracle_env_step(cfg, &envs[i], a, &out);
      sum += out.reward;
      if (out.terminated || out.truncated) {
        oracle_reset_draw(cfg, seed, (uint64_t)i, ep[i]++, i12, t3);
        oracle_env_reset(cfg, &envs[i], i12, t3, obs);
      }
    }
  return sum;
}

size_t oracle_sizeof_env(void) { return sizeof(OracleEnv); }
size_t oracle_sizeof_stepout(void) { return sizeof(OracleStepOut); }
size_t oracle_sizeof_cfg(void) { return sizeof(OracleCfg); }
