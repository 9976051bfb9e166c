/*
 * mpo.h -- C ABI of libmpo.so, the MI355X (gfx950) engine for mpi_opt's
 * trial-evaluation hot path.
 *
 * Conventions:
 *   - every function returns int status (MPO_OK = 0); the message of the last
 *     failure on the calling thread is mpo_last_error();
 *   - no exceptions cross the ABI;
 *   - the CALLER owns every device buffer (e.g. torch tensors' data_ptr());
 *     the library never allocates device memory: scratch comes from a caller
 *     workspace whose size is returned by the matching *_ws_bytes query;
 *   - every launching call takes an explicit hipStream_t (passed as void*) and
 *     only enqueues work: no host synchronisation, no allocation, so callers
 *     may capture any sequence of calls into a hipGraph;
 *   - not re-entrant per stream; thread-safe across streams/devices.  The
 *     population engines (mpo_pop_*, mpo_dn_*) fork part of a step onto side
 *     streams pooled per (device, caller stream): engines stepped from distinct
 *     caller streams never wait for each other's work.
 *
 * Row-major layouts throughout: matrix A(i,j) lives at A[i*ld + j].
 *
 * Each entry point cites the reference interface it replaces
 * (/root/reference/<file>:<line>).
 */
#ifndef MPO_H_
#define MPO_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPO_OK 0
#define MPO_EINVAL 1      /* bad argument (shape, null pointer, workspace too small) */
#define MPO_EHIP 2        /* HIP runtime error (launch failure, ...) */
#define MPO_ENOTSUP 3     /* shape outside what the kernels support */

/* Acquisition selection flags for mpo_gp_acq_score (skopt acquisition.py). */
#define MPO_ACQ_EI 1u     /* value = -EI  (skopt minimises -EI)  */
#define MPO_ACQ_PI 2u     /* value = -PI                         */
#define MPO_ACQ_LCB 4u    /* value = mu - kappa * sd             */

#define MPO_TOPK_MAX 8

const char* mpo_last_error(void);
/* Library version string, e.g. "mpo 0.1 gfx950". */
const char* mpo_version(void);

/* ------------------------------------------------------------------------
 * GP surrogate ("ask" hot path).
 * Replaces skopt.Optimizer.tell/ask's GaussianProcessRegressor fit tail and
 * _gaussian_acquisition, reached from Coordinator.fit (coordinator.py:63-79)
 * and Coordinator.ask (coordinator.py:46-50).
 * ---------------------------------------------------------------------- */

/* A prepared GP posterior (device pointers into the prepare workspace). */
typedef struct MpoGpModel {
    int32_t n;             /* observations                          */
    int32_t d;             /* dimensions                            */
    int32_t dp;            /* padded dimensions (4, 8, 16 or 32)    */
    int32_t np16;          /* n rounded up to 16                    */
    double amp;            /* ConstantKernel value                  */
    double y_mean;         /* normalize_y mean                      */
    double y_std;          /* normalize_y std                       */
    const double* xs;      /* [n][dp]  observations / length_scale  */
    const double* ls;      /* [dp]     length scales (pad = 1)      */
    const double* alpha;   /* [n]      K^-1 y_norm                  */
    const double* wfrag;   /* packed L^-1 MFMA B-fragments          */
    const double* L;       /* [n][n]   lower Cholesky factor        */
    const double* W;       /* [n][n]   L^-1 (lower)                 */
    int32_t* info;         /* device int: 0 ok, j+1 = chol failed at column j */
    const int32_t* wmeta;  /* per-wave B-stream plan of wfrag (scoring kernel) */
    const double* xb;      /* [np16+32][dp] (-2 xs, 1, |xs|^2, 0..) + a guard flag, or NULL:
                              the MFMA form of the candidate-observation distance,
                              set by mpo_gp_prepare when d + 2 <= dp; the flag is
                              the self-check's verdict (see mpo_gp_prepare) */
} MpoGpModel;

/* K(i,j) = amp * Matern52(|X_i/ls - X_j/ls|) + (i==j ? diag_add : 0).
 * X: [n][d] device, ls: [d] device, K: [n][ldk] device. */
int mpo_gp_kernel_matrix(const double* X, int n, int d, const double* ls, double amp,
                         double diag_add, double* K, int ldk, void* stream);

/* In-place lower Cholesky A = L L^T (upper triangle left untouched).
 * info (device int) = 0 on success, j+1 if the pivot of column j is <= 0. */
int mpo_chol_f64(double* A, int n, int lda, int32_t* info, void* stream);

/* Triangular solve with the lower factor L: trans=0 solves L X = B,
 * trans=1 solves L^T X = B; B [n][ldb] (nrhs columns) is overwritten with X. */
int mpo_trsm_f64(const double* L, int n, int lda, double* B, int nrhs, int ldb,
                 int trans, void* stream);

/* Workspace bytes for mpo_gp_prepare. */
size_t mpo_gp_prepare_ws_bytes(int n, int d);

/* Build a GP posterior from observations and fitted hyper-parameters:
 *   xs = X/ls;  K = amp*Matern52 + (noise + 1e-10 jitter) I;  L = chol(K);
 *   W = L^-1;  alpha = L^-T L^-1 y_norm;  pack W for the scoring kernel.
 * When d + 2 <= dp, model->xb is set and the scoring kernel may form
 * |c - x|^2 = |c|^2 + |x|^2 - 2 c.x on fp64 MFMA (absolute rounding error of a few
 * eps (|c|^2 + |x|^2) instead of the direct form's eps |c - x|^2).  The guard is
 * empirical, not a closed-form bound: (1) a device flag requires every |x/ls|^2 <= 2;
 * (2) a prepare-time self-check scores the model's own observations both ways --
 * r^2 = 0 on each one's own row and the smallest sd, the expansion's worst case --
 * and clears the flag unless (mu_n, q) agree within 1e-10 (q relative to
 * sd^2 = amp - q, mu_n relative to amp sum |alpha|); (3) per 16-candidate tile, the
 * expanded form is used only when every |c/ls|^2 <= 2.  Any other tile or model
 * takes the direct differences.  tests/test_gp_gpu.py checks the expanded path
 * against the exact posterior at 1e-9 on the fixtures and on a small-noise,
 * near-duplicate-observation problem.  MPO_GP_DIST=0 disables it.
 * X [n][d], y_norm [n], ls [d]: device.  `model` (host struct) receives
 * device pointers into `ws`, which must stay alive while the model is used.
 * Replaces GaussianProcessRegressor.fit's tail (sklearn _gpr.py:345-365) and
 * skopt's post-fit K_inv_ (skopt learning/gaussian_process/gpr.py). */
int mpo_gp_prepare(const double* X, const double* y_norm, int n, int d, const double* ls,
                   double amp, double noise, double y_mean, double y_std,
                   MpoGpModel* model, void* ws, size_t ws_bytes, void* stream);

/* Workspace bytes for mpo_gp_lml_grad (n <= 2048, d <= 32, batch thetas); 0 if unsupported. */
size_t mpo_gp_lml_ws_bytes(int n, int d, int batch);

/* Log-marginal likelihood and its gradient for `batch` hyper-parameter vectors at
 * once (one workgroup each): sklearn GaussianProcessRegressor(normalize_y=True,
 * alpha=1e-10).log_marginal_likelihood(theta, eval_gradient=True) for skopt's
 * kernel C * Matern(ls, nu=2.5) + WhiteKernel (sklearn _gpr.py:537-655), the
 * objective of the L-BFGS-B refit that skopt.Optimizer.tell runs from
 * Coordinator.fit (coordinator.py:63-79).
 *   X [n][d], y_norm [n] (normalised targets)      device
 *   theta [batch][d+2] = log[amp, ls_0..ls_{d-1}, noise]  (sklearn kernel.theta)
 *   lml [batch], grad [batch][d+2], info [batch]    device outputs
 * info[b] = j+1 when the Cholesky fails at column j: lml = -inf, grad = 0 (as
 * sklearn's LinAlgError branch); 0 otherwise. */
int mpo_gp_lml_grad(const double* X, const double* y_norm, int n, int d,
                    const double* theta, int batch, double* lml, double* grad,
                    int32_t* info, void* ws, size_t ws_bytes, void* stream);

/* Bytes of the device buffer mpo_gp_lml_grad_host stages through (d dims, batch thetas). */
size_t mpo_gp_lml_io_bytes(int d, int batch);

/* mpo_gp_lml_grad for one L-BFGS-B round of the refit with host-side input and
 * output: theta_host [batch][d+2] is copied into dev_io, the objective runs, and
 * out_host receives lml [batch] | grad [batch][d+2] | info (int32 [batch]) --
 * one call and one stream synchronisation per round instead of separate copies
 * (the refit runs ~100-200 rounds per fit, sklearn _gpr.py:296-337).  Pinned host
 * buffers avoid a staging copy.  Synchronises `stream`. */
int mpo_gp_lml_grad_host(const double* X, const double* y_norm, int n, int d,
                         const double* theta_host, int batch, double* out_host,
                         void* dev_io, size_t io_bytes, void* ws, size_t ws_bytes, void* stream);

/* Workspace bytes for mpo_gp_acq_score over m candidates. */
size_t mpo_gp_score_ws_bytes(const MpoGpModel* model, int64_t m, int k);

/* Score m candidates (transformed space, [m][d] device) under the posterior:
 *   mu, sd           : posterior mean / std (skopt predict(return_std=True));
 *   vals[a*m + i]    : minimised acquisition value for each flag a in
 *                      {EI, PI, LCB} order (rows for unset flags untouched);
 *   topk_idx/val[a*k + r] : the k smallest values of acquisition a, ties to the
 *                      lowest index (np.argsort(values)[:k] / np.argmin).
 * Any of mu, sd, vals may be NULL (not written).  topk arrays are device.
 * Replaces skopt _gaussian_acquisition + gaussian_ei/pi/lcb over the
 * n_points candidate sample, and the argsort/argmin that picks L-BFGS starts. */
int mpo_gp_acq_score(const MpoGpModel* model, const double* cand, int64_t m,
                     double y_opt, double xi, double kappa, unsigned flags,
                     double* mu, double* sd, double* vals, int k,
                     int64_t* topk_idx, double* topk_val,
                     void* ws, size_t ws_bytes, void* stream);

/* EI-only convenience (SURVEY §8b signature family): writes mu, sd, ei (= +EI)
 * and argmax (device int64, lowest index among maximal EI). */
int mpo_gp_ei_score(const MpoGpModel* model, const double* cand, int64_t m,
                    double y_opt, double xi, double* mu, double* sd, double* ei,
                    int64_t* argmax, void* ws, size_t ws_bytes, void* stream);

/* Acquisition value and gradient at `batch` points x [batch][d] (transformed
 * space, device): f[b] = the minimised value of acquisition acq[b] (device int32,
 * one of MPO_ACQ_EI / MPO_ACQ_PI / MPO_ACQ_LCB), g[b][d] its gradient.  The
 * objective of skopt's L-BFGS-B polish of the best candidates (skopt
 * gaussian_acquisition_1D with predict(return_mean_grad, return_std_grad)),
 * reached from Coordinator.ask (coordinator.py:46-50); one point per live
 * polish, all of an ask step's polishes in lockstep. */
int mpo_gp_acq_grad(const MpoGpModel* model, const double* x, int batch, const int32_t* acq,
                    double y_opt, double xi, double kappa, double* f, double* g, void* stream);

/* One polish round from the host: mpo_gp_acq_grad with x, acq, f, g in pinned
 * (hipHostMalloc / registered) host memory, read and written by the kernel in
 * place (no staging copies), then a synchronisation of `stream`.  MPO_EINVAL if
 * a buffer is not pinned host memory. */
int mpo_gp_acq_grad_host(const MpoGpModel* model, const double* x_host, int batch, const int32_t* acq_host,
                         double y_opt, double xi, double kappa, double* f_host, double* g_host, void* stream);

/* ------------------------------------------------------------------------
 * L-BFGS-B drivers (host C++, no Python in the loop).  skopt's refit runs
 * scipy.optimize.minimize(method="L-BFGS-B") from sklearn's
 * _constrained_optimization (_gpr.py:296-337) and its polish runs
 * fmin_l_bfgs_b(maxiter=20); both are reached from Coordinator.fit / ask
 * (coordinator.py:63-79, 46-50).  These run L-BFGS-B 3.0 with scipy's driver
 * rules over `nruns` independent starts whose objective evaluations are batched:
 * every round evaluates the point each live run needs in one call.  Outputs:
 * x_out [nruns][nvar], f_out [nruns] (scipy's OptimizeResult.fun), stats
 * [nruns][4] = (nit, nfev, status, 0) with status 1 = projected gradient <= gtol,
 * 2 = relative reduction <= ftol, 3 = maxiter, 4 = maxfun, 5 = abnormal line
 * search; *rounds = objective rounds.  bounds [nvar][2] = (lower, upper).
 * ---------------------------------------------------------------------- */
typedef struct MpoLbfgsbOptions {
    double ftol;        /* scipy ftol (factr * eps): minimize's default 2.22e-9, fmin_l_bfgs_b's 1e7 * eps */
    double gtol;        /* scipy gtol / pgtol (1e-5) */
    int32_t maxiter;    /* 15000 (minimize), 20 (skopt's polish) */
    int32_t maxfun;     /* 15000 */
    int32_t maxcor;     /* 10 */
    int32_t maxls;      /* 20 */
} MpoLbfgsbOptions;

/* Objective of mpo_lbfgsb_batched: f [batch], g [batch][nvar] at the points X
 * [batch][nvar] of runs ids [batch]; nonzero return aborts the minimisation. */
typedef int (*mpo_fg_batch_fn)(int batch, const double* X, const int32_t* ids, double* f, double* g, void* user);

/* The driver over a caller objective (host; the CPU tests compare it with scipy). */
int mpo_lbfgsb_batched(int nvar, int nruns, const double* x0, const double* bounds, const MpoLbfgsbOptions* opts,
                       mpo_fg_batch_fn fg, void* user, double* x_out, double* f_out, int32_t* stats,
                       int32_t* rounds);

/* A rendezvous for the concurrent refits on one device (the cl_min chains):
 * fits that share it evaluate their pending rounds together, one grouped launch
 * set per round of all registered fits, each theta's result unchanged.  Thread
 * safe; stats = grouped launch sets and the rounds they carried. */
int mpo_gp_lml_batcher_create(int device, void** handle);
int mpo_gp_lml_batcher_destroy(void* handle);
int mpo_gp_lml_batcher_stats(const void* handle, int64_t* launches, int64_t* rounds);

/* skopt's whole refit on the device objective: L-BFGS-B from starts [nruns][d+2]
 * (log theta) on -mpo_gp_lml_grad, one mpo_gp_lml_grad_host round per iteration
 * of all live runs (theta_host [nruns][d+2] and out_host as that call's pinned
 * buffers).  With a `batcher` (or NULL) of the stream's device, each round goes
 * through it and may launch together with other fits' rounds.  Replaces sklearn's
 * restart loop (_gpr.py:296-337) around scipy.optimize.minimize.  Synchronises
 * every round. */
int mpo_gp_fit_lml_host(const double* X, const double* y_norm, int n, int d, const double* starts, int nruns,
                        const double* bounds, const MpoLbfgsbOptions* opts, double* theta_host, double* out_host,
                        void* dev_io, size_t io_bytes, void* ws, size_t ws_bytes, double* x_out, double* f_out,
                        int32_t* stats, int32_t* rounds, void* batcher, void* stream);

/* skopt's polish of the best candidates: L-BFGS-B from starts [nruns][d] on the
 * minimised acquisition acq[r] of run r (mpo_gp_acq_grad_host rounds through the
 * pinned x_host [nruns][d], acq_host [nruns], f_host [nruns], g_host [nruns][d]).
 * Replaces skopt's fmin_l_bfgs_b(gaussian_acquisition_1D, x0, bounds, maxiter=20)
 * loop over the n_restarts_optimizer best candidates. */
int mpo_gp_polish_host(const MpoGpModel* model, const double* starts, const int32_t* acq, int nruns,
                       const double* bounds, const MpoLbfgsbOptions* opts, double y_opt, double xi, double kappa,
                       double* x_host, int32_t* acq_host, double* f_host, double* g_host, double* x_out,
                       double* f_out, int32_t* stats, int32_t* rounds, void* stream);

/* ------------------------------------------------------------------------
 * Population training of ragged MNIST-CNN trials.
 * Replaces ProcessBlock.train_model -> mpi_learn MPIKFoldManager.train()
 * (process_block.py:71-96) for test_mnist (mpiLAPI.py:138-176): every member
 * is one (trial, fold) pair; all members step together on one GPU.
 * ---------------------------------------------------------------------- */

/* One population member: the test_mnist hyper-parameters (option3:127-131)
 * plus the optimizer/dropout settings that the device table carries per trial. */
typedef struct MpoCnnSpec {
    int32_t nb_filters;   /* F      Integer(10, 50)  */
    int32_t kernel_size;  /* k      Integer(2, 10)   */
    int32_t pool_size;    /* p      Integer(2, 10)   */
    int32_t dense;        /* dense  Integer(50, 200) */
    float lr;             /* learning rate (reference: Adam, 1e-3)           */
    float dropout;        /* dropout rate (reference: 0.25, mpiLAPI.py:151)   */
    uint32_t seed;        /* dropout stream seed                             */
    int32_t options;      /* MPO_LOSS_* | MPO_OPT_* (0: the reference's binary_crossentropy + Adam) */
} MpoCnnSpec;

/* MpoCnnSpec.options: option3's --loss (hyperparameter_search_option3.py:61) and
 * master --optimizer (:60), both handed to mpi_learn's Algo (:270-275). */
#define MPO_LOSS_BCE 0x0      /* Keras binary_crossentropy on the softmax (mean over the 10 outputs) */
#define MPO_LOSS_CCE 0x1      /* Keras categorical_crossentropy (renormalised, clipped 1e-7)        */
#define MPO_LOSS_MASK 0xff
#define MPO_OPT_ADAM 0x000    /* Keras Adam (beta 0.9 / 0.999, eps 1e-8)                            */
#define MPO_OPT_SGD 0x100     /* Keras SGD, no momentum: p -= lr g                                  */
#define MPO_OPT_MASK 0xff00

typedef struct MpoPopSizes {
    int64_t n_params;     /* floats in the parameter arena (also grads, adam m, adam v) */
    int64_t act_floats;   /* floats in the activation arena                              */
    int64_t table_bytes;  /* device bytes for the member table + work lists              */
    int32_t n_members;
    int32_t batch;
} MpoPopSizes;

/* Plan a population (host only: layouts, ragged work lists).  *handle owns host
 * memory only; release with mpo_pop_destroy. */
int mpo_pop_create(const MpoCnnSpec* specs, int n_members, int batch, void** handle);
int mpo_pop_destroy(void* handle);
int mpo_pop_sizes(const void* handle, MpoPopSizes* out);
/* offsets[9] (floats into the parameter arena) of member's
 * w1 (k,k,1,F), b1, w2 (k,k,F,F), b2, w3 (s*s*F, dense), b3, w4 (dense,10), b4, end.
 * Keras weight shapes and order (Conv2D kernel (kh,kw,cin,cout), Dense (in,out)). */
int mpo_pop_param_layout(const void* handle, int member, int64_t* offsets);
/* offsets[15] (floats into the activation arena) of member's a1, a2, pd,
 * argmax (bytes at that float offset), h, hd, z3, dz3, dh, dp, dz2, dz1, w2t,
 * conv1 / conv2 weight-gradient partial slabs (diagnostics and tests). */
int mpo_pop_act_layout(const void* handle, int member, int64_t* offsets);
/* Bind caller-owned device arenas (zero-initialised by the caller) and upload
 * the work tables (async on `stream`). */
int mpo_pop_bind(void* handle, float* params, float* grads, float* adam_m, float* adam_v, float* act,
                 void* tables, void* stream);
/* One training step of every member on batch rows [row0, row0+batch) of its
 * sample order: sample = order[member*order_stride + row0 + b] indexes x
 * [n][784] f32 and labels [n] i32 (the k-fold split is this index gather).
 * step = global step counter (dropout stream; Adam t = step + 1).
 * loss_out[member] = mean Keras binary_crossentropy of the batch. */
int mpo_pop_train_step(void* handle, const float* x, const int32_t* labels, const int32_t* order,
                       int64_t order_stride, int64_t row0, int32_t step, float* loss_out, void* stream);
/* Validation forward (no dropout) of one batch: loss_sum[member] += sum of
 * per-sample losses, correct[member] += argmax hits. */
int mpo_pop_eval_step(void* handle, const float* x, const int32_t* labels, const int32_t* order,
                      int64_t order_stride, int64_t row0, float* loss_sum, int32_t* correct, void* stream);

/* Diagnostics: per-phase device milliseconds accumulated over the steps run
 * since the last reset, as "phase ms\n" lines into buf (cap bytes).  Only
 * populated when the plan was created with MPO_POP_PROFILE=1 in the
 * environment (then every step ends in an event sync); returns MPO_ENOTSUP
 * otherwise.  reset != 0 clears the accumulators after the read. */
int mpo_pop_profile(void* handle, char* buf, size_t cap, int reset);

/* ------------------------------------------------------------------------
 * DenseNet population (BASELINE config 5).
 * Replaces the per-block Keras training of DenseNet (densenet.py:135-196, built
 * by base_model.py:61-72 / mpiLAPI.py:197-201, trained by process_block.py:71-96).
 * All members share one architecture (the reference grid searches lr only,
 * base_model.py:84-92); each member has its own lr, weights and sample order.
 * ---------------------------------------------------------------------- */
typedef struct MpoDnArch {
    int32_t H, W, C;          /* img_dim (channels last)                 */
    int32_t classes;          /* nb_classes                              */
    int32_t depth;            /* 3 N + 4                                 */
    int32_t nb_dense_block;
    int32_t growth;           /* growth_rate                             */
    int32_t nb_filter;
} MpoDnArch;

typedef struct MpoDnSizes {
    int64_t n_params;     /* floats per member in the parameter arena (also grads, adam m, v) */
    int64_t n_state;      /* floats per member of BN moving statistics                         */
    int64_t act_floats;   /* floats in the activation arena (all members)                      */
    int32_t n_members;
    int32_t batch;
    int32_t n_layers;
    int32_t reserved;
} MpoDnSizes;

int mpo_dn_create(const MpoDnArch* arch, int n_members, int batch, void** handle);
int mpo_dn_destroy(void* handle);
int mpo_dn_sizes(const void* handle, MpoDnSizes* out);
/* Layer i: geom[8] = kind (0 initial conv, 1 dense-block conv, 2 transition, 3 head),
 * stage, H, W, cin, cout, kernel size, concat channel offset; offs[6] = float
 * offsets within a member's parameter block of the conv kernel (head: dense kernel),
 * gamma, beta, and within its state block of moving mean, moving variance, and
 * (head only) the dense bias; -1 where absent.  Keras shapes: conv (ks,ks,cin,cout),
 * gamma/beta/moving stats [H] (BatchNormalization axis=1 of NHWC). */
int mpo_dn_layer(const void* handle, int i, int32_t* geom, int64_t* offs);
/* Bind caller-owned, zero-initialised device arenas: params/grads/adam_m/adam_v
 * [n_members][n_params], state [n_members][n_state], act [act_floats]; lr is a
 * HOST array of n_members learning rates (copied, stream-synchronised). */
int mpo_dn_bind(void* handle, float* params, float* grads, float* adam_m, float* adam_v, float* state, float* act,
                const float* lr, void* stream);
/* One Adam step of every member on rows [row0, row0+batch) of its order table:
 * sample = order[member*order_stride + row0 + b] into x [n][H][W][C] f32, labels
 * [n] i32.  BN uses batch statistics and updates the moving averages.
 * loss_out[member] = mean categorical CE + l2 penalty (before the update);
 * Adam t = step + 1. */
int mpo_dn_train_step(void* handle, const float* x, const int32_t* labels, const int32_t* order,
                      int64_t order_stride, int64_t row0, int32_t step, float* loss_out, void* stream);
/* Inference-mode forward (BN moving averages) of one batch: loss_sum[member] +=
 * sum of per-sample CE, correct[member] += argmax hits. */
int mpo_dn_eval_step(void* handle, const float* x, const int32_t* labels, const int32_t* order,
                     int64_t order_stride, int64_t row0, float* loss_sum, int32_t* correct, void* stream);
/* out[member] = 1e-4 * sum of squared parameters (Keras adds it to val_loss). */
int mpo_dn_penalty(void* handle, float* out, void* stream);

/* k-fold index gather: out[r][:] = X[idx[r]][:] (the fold split
 * that mpi_learn does with per-fold communicators becomes an index gather). */
int mpo_kfold_gather(const float* X, const int32_t* idx, int64_t rows, int row_elems, float* out,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPO_H_ */
