// lbfgsb.cpp -- L-BFGS-B on the host, batched over independent runs whose
// objective is evaluated on the GPU, with no Python in the loop.
//
// skopt's refit (sklearn GaussianProcessRegressor._constrained_optimization,
// _gpr.py:296-337 -> scipy.optimize.minimize(method="L-BFGS-B", jac=True)) and its
// acquisition polish (skopt Optimizer._ask -> fmin_l_bfgs_b(maxiter=20)) are
// L-BFGS-B runs over a device objective, reached from Coordinator.fit / ask
// (/root/reference/coordinator.py:63-79, 46-50).  gp_fit.lbfgsb_batched drives
// scipy's setulb from Python; every round then holds the GIL for ~18 us per three
// runs, which caps one process at ~200-260 refits/s however many cl_min chains
// run (r05, profiles/r05/lbfgs_host_and_chain_g.log).  Here the same algorithm
// runs in C++ behind one ctypes call per fit (ctypes releases the GIL), so
// concurrent chains overlap their host work as well as their device rounds.
//
// The algorithm is L-BFGS-B 3.0 (Byrd, Lu, Nocedal, Zhu, SIAM J. Sci. Comput. 16
// (1995); Morales, Nocedal, ACM TOMS 38 (2011)), as scipy 1.15's setulb runs it:
// generalized Cauchy point over the sorted breakpoints, direct primal subspace
// minimisation with the projection / backtracking step of 3.0, the Moré-Thuente
// line search (dcsrch: ftol 1e-3, gtol 0.9, xtol 0.1) with at most maxls trial
// steps, the same restarts of the limited memory on a failed factorisation or
// line search, and the same stopping tests (projected gradient <= pgtol, relative
// reduction <= factr * eps), plus scipy's driver rules (maxiter counted on
// NEW_X, maxfun on objective evaluations, one evaluation reused when the same x
// is requested twice -- ScalarFunction's cache).  The middle matrix of the
// subspace step (formk) is formed from the current free set on every call
// rather than updated incrementally; in exact arithmetic that is the same
// matrix, so iterates agree with scipy's to rounding (tests/test_lbfgsb.py
// compares them on the GP objective and on bound-constrained test functions).
//
// Provenance and licence.  The routines below are a C++ translation of two
// BSD-licensed Fortran packages, following their structure and variable names:
//   * L-BFGS-B 3.0 (cauchy, subsm, formk/bmv, the heap sort of the breakpoints,
//     and the LINPACK dpofa / dtrsl factor-and-solve it calls), distributed under
//     the "New BSD License":
//       Copyright (c) 2011 Ciyou Zhu, Richard Byrd, Jorge Nocedal and Jose Luis
//       Morales.  All rights reserved.
//   * the line search dcsrch / dcstep (Jorge J. More and David J. Thuente,
//     MINPACK-1 Project, Argonne National Laboratory; MINPACK-2 Project,
//     Argonne National Laboratory and University of Minnesota: Brett M.
//     Averick, Richard G. Carter and Jorge J. More), shipped inside the
//     L-BFGS-B 3.0 distribution and covered by the notice below.
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are met:
//   (1) redistributions of source code must retain the above copyright notice,
//   this list of conditions and the following disclaimer; (2) redistributions in
//   binary form must reproduce the above copyright notice, this list of
//   conditions and the following disclaimer in the documentation and/or other
//   materials provided with the distribution; (3) neither the name of the
//   copyright holders nor the names of its contributors may be used to endorse
//   or promote products derived from this software without specific prior
//   written permission.  THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND
//   CONTRIBUTORS "AS IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT
//   NOT LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A
//   PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT HOLDERS
//   OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL,
//   EXEMPLARY, OR CONSEQUENTIAL DAMAGES ARISING IN ANY WAY OUT OF THE USE OF
//   THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#pragma clang fp contract(off)
// max / min of doubles are fmax / fmin throughout: a NaN operand yields the other one, as
// the scipy build's L-BFGS-B does -- an infinite objective value (sklearn's LinAlgError
// branch: -LML = +inf) turns the cubic step of dcstep into NaN, which then clamps to the
// step bounds instead of propagating (tests/test_lbfgsb.py::test_infinite_objective_*).

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mpo_internal.h"

namespace {

inline double ddot(int n, const double* a, const double* b) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

// Moré-Thuente safeguarded step (MINPACK-2 dcstep)
void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy, double& stp, double fp, double dp,
            bool& brackt, double stpmin, double stpmax) {
    const double sgnd = dp * (dx / std::fabs(dx));
    double stpf;
    if (fp > fx) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = std::fmax(std::fmax(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
        double gamma = s * std::sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp < stx) gamma = -gamma;
        const double p = (gamma - dx) + theta;
        const double q = ((gamma - dx) + gamma) + dp;
        const double r = p / q;
        const double stpc = stx + r * (stp - stx);
        const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
        if (std::fabs(stpc - stx) < std::fabs(stpq - stx)) stpf = stpc;
        else stpf = stpc + (stpq - stpc) / 2.0;
        brackt = true;
    } else if (sgnd < 0.0) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = std::fmax(std::fmax(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
        double gamma = s * std::sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = ((gamma - dp) + gamma) + dx;
        const double r = p / q;
        const double stpc = stp + r * (stx - stp);
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
        brackt = true;
    } else if (std::fabs(dp) < std::fabs(dx)) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = std::fmax(std::fmax(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
        double gamma = s * std::sqrt(std::fmax(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = (gamma + (dx - dp)) + gamma;
        const double r = p / q;
        double stpc;
        if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
        else if (stp > stx) stpc = stpmax;
        else stpc = stpmin;
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        if (brackt) {
            stpf = std::fabs(stpc - stp) < std::fabs(stpq - stp) ? stpc : stpq;
            if (stp > stx) stpf = std::fmin(stp + 0.66 * (sty - stp), stpf);
            else stpf = std::fmax(stp + 0.66 * (sty - stp), stpf);
        } else {
            stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
            stpf = std::fmin(stpmax, stpf);
            stpf = std::fmax(stpmin, stpf);
        }
    } else {
        if (brackt) {
            const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
            const double s = std::fmax(std::fmax(std::fabs(theta), std::fabs(dy)), std::fabs(dp));
            double gamma = s * std::sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
            if (stp > sty) gamma = -gamma;
            const double p = (gamma - dp) + theta;
            const double q = ((gamma - dp) + gamma) + dy;
            const double r = p / q;
            stpf = stp + r * (sty - stp);
        } else if (stp > stx) {
            stpf = stpmax;
        } else {
            stpf = stpmin;
        }
    }
    if (fp > fx) {
        sty = stp; fy = fp; dy = dp;
    } else {
        if (sgnd < 0.0) { sty = stx; fy = fx; dy = dx; }
        stx = stp; fx = fp; dx = dp;
    }
    stp = stpf;
}

// Moré-Thuente line search (MINPACK-2 dcsrch) in reverse communication; the state
// persists across searches as the Fortran save arrays do.
struct Dcsrch {
    enum Task { START, FG, CONV, WARN, ERROR };
    Task task = START;
    bool brackt = false;
    int stage = 1;
    double ginit = 0, gtest = 0, gx = 0, gy = 0, finit = 0, fx = 0, fy = 0, stx = 0, sty = 0, stmin = 0, stmax = 0,
           width = 0, width1 = 0;

    void step(double f, double g, double& stp, double ftol, double gtol, double xtol, double stpmin, double stpmax) {
        if (task == START) {
            if (stp < stpmin || stp > stpmax || g >= 0.0 || ftol < 0.0 || gtol < 0.0 || xtol < 0.0 || stpmin < 0.0 ||
                stpmax < stpmin) {
                task = ERROR;
                return;
            }
            brackt = false;
            stage = 1;
            finit = f;
            ginit = g;
            gtest = ftol * ginit;
            width = stpmax - stpmin;
            width1 = width / 0.5;
            stx = 0.0; fx = finit; gx = ginit;
            sty = 0.0; fy = finit; gy = ginit;
            stmin = 0.0;
            stmax = stp + 4.0 * stp;
            task = FG;
            return;
        }
        const double ftest = finit + stp * gtest;
        if (stage == 1 && f <= ftest && g >= 0.0) stage = 2;
        if (brackt && (stp <= stmin || stp >= stmax)) task = WARN;
        if (brackt && stmax - stmin <= xtol * stmax) task = WARN;
        if (stp == stpmax && f <= ftest && g <= gtest) task = WARN;
        if (stp == stpmin && (f > ftest || g >= gtest)) task = WARN;
        if (f <= ftest && std::fabs(g) <= gtol * (-ginit)) task = CONV;
        if (task == WARN || task == CONV) return;
        if (stage == 1 && f <= fx && f > ftest) {
            const double fm = f - stp * gtest;
            double fxm = fx - stx * gtest, fym = fy - sty * gtest;
            const double gm = g - gtest;
            double gxm = gx - gtest, gym = gy - gtest;
            dcstep(stx, fxm, gxm, sty, fym, gym, stp, fm, gm, brackt, stmin, stmax);
            fx = fxm + stx * gtest;
            fy = fym + sty * gtest;
            gx = gxm + gtest;
            gy = gym + gtest;
        } else {
            dcstep(stx, fx, gx, sty, fy, gy, stp, f, g, brackt, stmin, stmax);
        }
        if (brackt) {
            if (std::fabs(sty - stx) >= 0.66 * width1) stp = stx + 0.5 * (sty - stx);
            width1 = width;
            width = std::fabs(sty - stx);
        }
        if (brackt) {
            stmin = std::fmin(stx, sty);
            stmax = std::fmax(stx, sty);
        } else {
            stmin = stp + 1.1 * (stp - stx);
            stmax = stp + 4.0 * (stp - stx);
        }
        stp = std::fmax(stp, stpmin);
        stp = std::fmin(stp, stpmax);
        if ((brackt && (stp <= stmin || stp >= stmax)) || (brackt && stmax - stmin <= xtol * stmax)) stp = stx;
        task = FG;
    }
};

enum Status : int32_t {
    kRunning = 0,
    kConvPgtol = 1,     // CONVERGENCE: NORM_OF_PROJECTED_GRADIENT_<=_PGTOL
    kConvFactr = 2,     // CONVERGENCE: REL_REDUCTION_OF_F_<=_FACTR*EPSMCH
    kStopMaxiter = 3,   // STOP: TOTAL NO. OF ITERATIONS REACHED LIMIT (scipy driver)
    kStopMaxfun = 4,    // STOP: TOTAL NO. OF f AND g EVALUATIONS EXCEEDS LIMIT (scipy driver)
    kAbnormal = 5,      // ABNORMAL_TERMINATION_IN_LNSRCH
};

// One L-BFGS-B minimisation.  Matrices are column-major with 1-based accessors,
// as the published algorithm indexes them.
class Lbfgsb {
  public:
    Lbfgsb(int n, const double* lo, const double* hi, const int* nbd, double factr, double pgtol, int m, int maxls,
           int maxiter, int maxfun)
        : n_(n), m_(m), maxls_(maxls), maxiter_(maxiter), maxfun_(maxfun), l_(lo), u_(hi), nbd_(nbd), pgtol_(pgtol) {
        epsmch_ = 2.220446049250313e-16;
        tol_ = factr * epsmch_;
        x_.assign(n, 0.0); g_.assign(n, 0.0); z_.assign(n, 0.0); r_.assign(n, 0.0); d_.assign(n, 0.0);
        t_.assign(n, 0.0); xp_.assign(n, 0.0);
        ws_.assign((size_t)n * m, 0.0); wy_.assign((size_t)n * m, 0.0);
        sy_.assign((size_t)m * m, 0.0); ss_.assign((size_t)m * m, 0.0); wt_.assign((size_t)m * m, 0.0);
        wn_.assign((size_t)4 * m * m, 0.0);
        wa_.assign((size_t)8 * m, 0.0);
        wv_.assign((size_t)2 * m, 0.0);
        index_.assign(n, 0); iwhere_.assign(n, 0); indx2_.assign(n, 0);
        nfree_ = n;
    }

    // x0 already clipped into the bounds (scipy: np.clip); evaluate at x() next.
    void start(const double* x0) {
        std::copy(x0, x0 + n_, x_.begin());
        active();
        phase_ = kPhaseStart;
    }
    const double* x() const { return x_.data(); }
    int status() const { return status_; }
    int nit() const { return nit_; }
    int nfev() const { return nfev_; }
    void count_evaluation() { ++nfev_; }

    // f, g at x(): returns true when the next f, g at x() are needed, false when done.
    bool deliver(double f, const double* g) {
        f_ = f;
        std::copy(g, g + n_, g_.begin());
        if (phase_ == kPhaseStart) {
            sbgnrm_ = projgr();
            if (sbgnrm_ <= pgtol_) return finish(kConvPgtol);
            return iterate();
        }
        return linesearch(false);
    }

  private:
    enum Phase { kPhaseStart, kPhaseLnsrch };
    // 1-based accessors
    double& WS(int i, int j) { return ws_[(size_t)(j - 1) * n_ + (i - 1)]; }
    double& WY(int i, int j) { return wy_[(size_t)(j - 1) * n_ + (i - 1)]; }
    double& SY(int i, int j) { return sy_[(size_t)(j - 1) * m_ + (i - 1)]; }
    double& SS(int i, int j) { return ss_[(size_t)(j - 1) * m_ + (i - 1)]; }
    double& WT(int i, int j) { return wt_[(size_t)(j - 1) * m_ + (i - 1)]; }
    double& WN(int i, int j) { return wn_[(size_t)(j - 1) * 2 * m_ + (i - 1)]; }
    int nxt(int p) const { return p % m_ + 1; }

    bool finish(Status s) {
        status_ = s;
        return false;
    }

    void reset_memory() {
        info_ = 0; col_ = 0; head_ = 1; theta_ = 1.0; iupdat_ = 0; updatd_ = false;
    }

    void active() {
        cnstnd_ = false;
        boxed_ = true;
        for (int i = 0; i < n_; ++i) {
            if (nbd_[i] > 0) {
                if (nbd_[i] <= 2 && x_[i] <= l_[i]) {
                    if (x_[i] < l_[i]) x_[i] = l_[i];
                } else if (nbd_[i] >= 2 && x_[i] >= u_[i]) {
                    if (x_[i] > u_[i]) x_[i] = u_[i];
                }
            }
        }
        for (int i = 0; i < n_; ++i) {
            if (nbd_[i] != 2) boxed_ = false;
            if (nbd_[i] == 0) {
                iwhere_[i] = -1;
            } else {
                cnstnd_ = true;
                iwhere_[i] = (nbd_[i] == 2 && u_[i] - l_[i] <= 0.0) ? 3 : 0;
            }
        }
    }

    double projgr() const {
        double s = 0.0;
        for (int i = 0; i < n_; ++i) {
            double gi = g_[i];
            if (nbd_[i] != 0) {
                if (gi < 0.0) {
                    if (nbd_[i] >= 2) gi = std::fmax(x_[i] - u_[i], gi);
                } else {
                    if (nbd_[i] <= 2) gi = std::fmin(x_[i] - l_[i], gi);
                }
            }
            s = std::fmax(s, std::fabs(gi));
        }
        return s;
    }

    // LINPACK dpofa on the leading n x n of a (column-major, leading dimension lda):
    // A = R^T R with R in the upper triangle; 0 or the failing column (1-based)
    static int dpofa(double* a, int lda, int n) {
        auto A = [&](int i, int j) -> double& { return a[(size_t)(j - 1) * lda + (i - 1)]; };
        for (int j = 1; j <= n; ++j) {
            double s = 0.0;
            for (int k = 1; k <= j - 1; ++k) {
                double t = A(k, j) - ddot(k - 1, &A(1, k), &A(1, j));
                t = t / A(k, k);
                A(k, j) = t;
                s += t * t;
            }
            s = A(j, j) - s;
            if (s <= 0.0) return j;
            A(j, j) = std::sqrt(s);
        }
        return 0;
    }

    // LINPACK dtrsl for an upper triangular T: job 1 solves T x = b, job 11 T^T x = b
    static int dtrsl(double* t, int ldt, int n, double* b, int job) {
        auto T = [&](int i, int j) -> double& { return t[(size_t)(j - 1) * ldt + (i - 1)]; };
        for (int k = 1; k <= n; ++k)
            if (T(k, k) == 0.0) return k;
        if (job == 1) {
            b[n - 1] = b[n - 1] / T(n, n);
            for (int jj = 2; jj <= n; ++jj) {
                const int j = n - jj + 1;
                const double temp = -b[j];
                for (int i = 1; i <= j; ++i) b[i - 1] += temp * T(i, j + 1);
                b[j - 1] = b[j - 1] / T(j, j);
            }
        } else {
            b[0] = b[0] / T(1, 1);
            for (int j = 2; j <= n; ++j) {
                b[j - 1] = b[j - 1] - ddot(j - 1, &T(1, j), b);
                b[j - 1] = b[j - 1] / T(j, j);
            }
        }
        return 0;
    }

    // product of the 2col x 2col middle matrix of the compact L-BFGS form with v
    int bmv(const double* v, double* p) {
        const int col = col_;
        if (col == 0) return 0;
        p[col] = v[col];
        for (int i = 2; i <= col; ++i) {
            const int i2 = col + i;
            double sum = 0.0;
            for (int k = 1; k <= i - 1; ++k) sum += SY(i, k) * v[k - 1] / SY(k, k);
            p[i2 - 1] = v[i2 - 1] + sum;
        }
        if (dtrsl(wt_.data(), m_, col, p + col, 11)) return -1;
        for (int i = 1; i <= col; ++i) p[i - 1] = v[i - 1] / std::sqrt(SY(i, i));
        if (dtrsl(wt_.data(), m_, col, p + col, 1)) return -1;
        for (int i = 1; i <= col; ++i) p[i - 1] = -p[i - 1] / std::sqrt(SY(i, i));
        for (int i = 1; i <= col; ++i) {
            double sum = 0.0;
            for (int k = i + 1; k <= col; ++k) sum += SY(k, i) * p[col + k - 1] / SY(i, i);
            p[i - 1] += sum;
        }
        return 0;
    }

    // heap of the breakpoints t[0..nn): iheap == 0 builds it; then the least moves to t[nn-1]
    static void hpsolb(int nn, double* t, int* iorder, int iheap) {
        auto T = [&](int i) -> double& { return t[i - 1]; };
        auto O = [&](int i) -> int& { return iorder[i - 1]; };
        if (iheap == 0) {
            for (int k = 2; k <= nn; ++k) {
                const double ddum = T(k);
                const int indxin = O(k);
                int i = k;
                while (i > 1) {
                    const int j = i / 2;
                    if (ddum < T(j)) {
                        T(i) = T(j); O(i) = O(j); i = j;
                    } else {
                        break;
                    }
                }
                T(i) = ddum; O(i) = indxin;
            }
        }
        if (nn > 1) {
            int i = 1;
            const double out = T(1);
            const int indxou = O(1);
            const double ddum = T(nn);
            const int indxin = O(nn);
            for (;;) {
                int j = i + i;
                if (j <= nn - 1) {
                    if (T(j + 1) < T(j)) j = j + 1;
                    if (T(j) < ddum) {
                        T(i) = T(j); O(i) = O(j); i = j;
                        continue;
                    }
                }
                break;
            }
            T(i) = ddum; O(i) = indxin;
            T(nn) = out; O(nn) = indxou;
        }
    }

    // generalized Cauchy point z along the projected steepest descent path
    int cauchy() {
        const int n = n_, m = m_, col = col_, col2 = 2 * col;
        double* p = wa_.data();
        double* c = wa_.data() + 2 * m;
        double* wbp = wa_.data() + 4 * m;
        double* v = wa_.data() + 6 * m;
        double* t = t_.data();          // breakpoints (the line search's t is set after this)
        double* d = d_.data();
        int* iorder = indx2_.data();
        if (sbgnrm_ <= 0.0) {
            z_ = x_;
            return 0;
        }
        bool bnded = true;
        int nfree = n + 1, nbreak = 0, ibkmin = 0;
        double bkmin = 0.0, f1 = 0.0, tl = 0.0, tu = 0.0;
        for (int i = 0; i < col2; ++i) p[i] = 0.0;
        for (int i = 1; i <= n; ++i) {
            const double neggi = -g_[i - 1];
            const int nb = nbd_[i - 1];
            int& iw = iwhere_[i - 1];
            if (iw != 3 && iw != -1) {
                if (nb <= 2) tl = x_[i - 1] - l_[i - 1];
                if (nb >= 2) tu = u_[i - 1] - x_[i - 1];
                const bool xlower = nb <= 2 && tl <= 0.0;
                const bool xupper = nb >= 2 && tu <= 0.0;
                iw = 0;
                if (xlower) {
                    if (neggi <= 0.0) iw = 1;
                } else if (xupper) {
                    if (neggi >= 0.0) iw = 2;
                } else {
                    if (std::fabs(neggi) <= 0.0) iw = -3;
                }
            }
            int pointr = head_;
            if (iw != 0 && iw != -1) {
                d[i - 1] = 0.0;
            } else {
                d[i - 1] = neggi;
                f1 -= neggi * neggi;
                for (int j = 1; j <= col; ++j) {
                    p[j - 1] += WY(i, pointr) * neggi;
                    p[col + j - 1] += WS(i, pointr) * neggi;
                    pointr = nxt(pointr);
                }
                if (nb <= 2 && nb != 0 && neggi < 0.0) {
                    ++nbreak;
                    iorder[nbreak - 1] = i;
                    t[nbreak - 1] = tl / (-neggi);
                    if (nbreak == 1 || t[nbreak - 1] < bkmin) { bkmin = t[nbreak - 1]; ibkmin = nbreak; }
                } else if (nb >= 2 && neggi > 0.0) {
                    ++nbreak;
                    iorder[nbreak - 1] = i;
                    t[nbreak - 1] = tu / neggi;
                    if (nbreak == 1 || t[nbreak - 1] < bkmin) { bkmin = t[nbreak - 1]; ibkmin = nbreak; }
                } else {
                    --nfree;
                    iorder[nfree - 1] = i;
                    if (std::fabs(neggi) > 0.0) bnded = false;
                }
            }
        }
        if (theta_ != 1.0)
            for (int j = 0; j < col; ++j) p[col + j] *= theta_;
        z_ = x_;
        if (nbreak == 0 && nfree == n + 1) return 0;
        for (int j = 0; j < col2; ++j) c[j] = 0.0;
        double f2 = -theta_ * f1;
        const double f2_org = f2;
        if (col > 0) {
            if (bmv(p, v)) return -1;
            f2 -= ddot(col2, v, p);
        }
        double dtm = -f1 / f2;
        double tsum = 0.0;
        nseg_ = 1;
        bool located = nbreak == 0;   // go straight to the GCP
        if (!located) {
            int nleft = nbreak, iter = 1;
            double tj = 0.0;
            for (;;) {
                const double tj0 = tj;
                int ibp;
                if (iter == 1) {
                    tj = bkmin;
                    ibp = iorder[ibkmin - 1];
                } else {
                    if (iter == 2) {
                        if (ibkmin != nbreak) {
                            t[ibkmin - 1] = t[nbreak - 1];
                            iorder[ibkmin - 1] = iorder[nbreak - 1];
                        }
                    }
                    hpsolb(nleft, t, iorder, iter - 2);
                    tj = t[nleft - 1];
                    ibp = iorder[nleft - 1];
                }
                const double dt = tj - tj0;
                if (dtm < dt) break;     // the minimiser lies in this interval
                tsum += dt;
                --nleft;
                ++iter;
                const double dibp = d[ibp - 1];
                d[ibp - 1] = 0.0;
                double zibp;
                if (dibp > 0.0) {
                    zibp = u_[ibp - 1] - x_[ibp - 1];
                    z_[ibp - 1] = u_[ibp - 1];
                    iwhere_[ibp - 1] = 2;
                } else {
                    zibp = l_[ibp - 1] - x_[ibp - 1];
                    z_[ibp - 1] = l_[ibp - 1];
                    iwhere_[ibp - 1] = 1;
                }
                if (nleft == 0 && nbreak == n) {
                    // every variable is fixed: z is the GCP
                    dtm = dt;
                    if (col > 0)
                        for (int j = 0; j < col2; ++j) c[j] += dtm * p[j];
                    return 0;
                }
                ++nseg_;
                const double dibp2 = dibp * dibp;
                f1 = f1 + dt * f2 + dibp2 - theta_ * dibp * zibp;
                f2 = f2 - theta_ * dibp2;
                if (col > 0) {
                    for (int j = 0; j < col2; ++j) c[j] += dt * p[j];
                    int pointr = head_;
                    for (int j = 1; j <= col; ++j) {
                        wbp[j - 1] = WY(ibp, pointr);
                        wbp[col + j - 1] = theta_ * WS(ibp, pointr);
                        pointr = nxt(pointr);
                    }
                    if (bmv(wbp, v)) return -1;
                    const double wmc = ddot(col2, c, v);
                    const double wmp = ddot(col2, p, v);
                    const double wmw = ddot(col2, wbp, v);
                    for (int j = 0; j < col2; ++j) p[j] += -dibp * wbp[j];
                    f1 += dibp * wmc;
                    f2 += 2.0 * dibp * wmp - dibp2 * wmw;
                }
                f2 = std::fmax(epsmch_ * f2_org, f2);
                if (nleft > 0) {
                    dtm = -f1 / f2;
                    continue;
                } else if (bnded) {
                    f1 = 0.0; f2 = 0.0; dtm = 0.0;
                } else {
                    dtm = -f1 / f2;
                }
                break;
            }
        }
        if (dtm <= 0.0) dtm = 0.0;
        tsum += dtm;
        for (int i = 0; i < n; ++i) z_[i] += tsum * d[i];
        if (col > 0)
            for (int j = 0; j < col2; ++j) c[j] += dtm * p[j];
        return 0;
    }

    // free / active sets at the GCP and the variables entering / leaving the free set
    void freev() {
        const int n = n_;
        nenter_ = 0;
        ileave_ = n + 1;
        if (iter_ > 0 && cnstnd_) {
            for (int i = 1; i <= nfree_; ++i) {
                const int k = index_[i - 1];
                if (iwhere_[k - 1] > 0) { --ileave_; indx2_[ileave_ - 1] = k; }
            }
            for (int i = 1 + nfree_; i <= n; ++i) {
                const int k = index_[i - 1];
                if (iwhere_[k - 1] <= 0) { ++nenter_; indx2_[nenter_ - 1] = k; }
            }
        }
        wrk_ = (ileave_ < n + 1) || (nenter_ > 0) || updatd_;
        nfree_ = 0;
        int iact = n + 1;
        for (int i = 1; i <= n; ++i) {
            if (iwhere_[i - 1] <= 0) { ++nfree_; index_[nfree_ - 1] = i; }
            else { --iact; index_[iact - 1] = i; }
        }
    }

    // the factorised middle matrix K of the subspace step, from the current free set
    int formk() {
        const int col = col_, nsub = nfree_;
        std::vector<double> yy((size_t)col * col), sa((size_t)col * col), sy2((size_t)col * col);
        auto YY = [&](int i, int j) -> double& { return yy[(size_t)(j - 1) * col + (i - 1)]; };
        auto SA = [&](int i, int j) -> double& { return sa[(size_t)(j - 1) * col + (i - 1)]; };
        auto SYZ = [&](int i, int j) -> double& { return sy2[(size_t)(j - 1) * col + (i - 1)]; };
        auto ptr = [&](int j) { int p = head_ + j - 1; return p > m_ ? p - m_ : p; };
        for (int iy = 1; iy <= col; ++iy) {
            const int ip = ptr(iy);
            for (int jy = 1; jy <= iy; ++jy) {
                const int jp = ptr(jy);
                double t1 = 0.0, t2 = 0.0;
                for (int k = 1; k <= nsub; ++k) { const int k1 = index_[k - 1]; t1 += WY(k1, ip) * WY(k1, jp); }
                for (int k = nsub + 1; k <= n_; ++k) { const int k1 = index_[k - 1]; t2 += WS(k1, ip) * WS(k1, jp); }
                YY(iy, jy) = t1;     // Y' Z Z' Y (free variables)
                SA(iy, jy) = t2;     // S' A A' S (active variables)
            }
        }
        for (int is = 1; is <= col; ++is) {
            const int ip = ptr(is);
            for (int jy = 1; jy <= col; ++jy) {
                const int jp = ptr(jy);
                double t = 0.0;
                if (is <= jy) {      // R_z: upper triangle of S' Z Z' Y
                    for (int k = 1; k <= nsub; ++k) { const int k1 = index_[k - 1]; t += WS(k1, ip) * WY(k1, jp); }
                } else {             // L_a: strictly lower triangle of S' A A' Y
                    for (int k = nsub + 1; k <= n_; ++k) { const int k1 = index_[k - 1]; t += WS(k1, ip) * WY(k1, jp); }
                }
                SYZ(is, jy) = t;
            }
        }
        for (int iy = 1; iy <= col; ++iy) {
            const int is = col + iy;
            for (int jy = 1; jy <= iy; ++jy) {
                const int js = col + jy;
                WN(jy, iy) = YY(iy, jy) / theta_;
                WN(js, is) = SA(iy, jy) * theta_;
            }
            for (int jy = 1; jy <= iy - 1; ++jy) WN(jy, is) = -SYZ(iy, jy);
            for (int jy = iy; jy <= col; ++jy) WN(jy, is) = SYZ(iy, jy);
            WN(iy, iy) += SY(iy, iy);
        }
        const int m2 = 2 * m_;
        if (dpofa(wn_.data(), m2, col)) return -1;
        const int col2 = 2 * col;
        for (int js = col + 1; js <= col2; ++js)
            if (dtrsl(wn_.data(), m2, col, &WN(1, js), 11)) return -1;
        for (int is = col + 1; is <= col2; ++is)
            for (int js = is; js <= col2; ++js) WN(is, js) += ddot(col, &WN(1, is), &WN(1, js));
        if (dpofa(&WN(col + 1, col + 1), m2, col)) return -2;
        return 0;
    }

    // r = -Z'(B (z - x) + g) over the free variables
    int cmprlb() {
        const int col = col_;
        if (!cnstnd_ && col > 0) {
            for (int i = 0; i < n_; ++i) r_[i] = -g_[i];
            return 0;
        }
        for (int i = 1; i <= nfree_; ++i) {
            const int k = index_[i - 1];
            r_[i - 1] = -theta_ * (z_[k - 1] - x_[k - 1]) - g_[k - 1];
        }
        double* wa = wa_.data();
        if (bmv(wa + 2 * m_, wa)) return -8;
        int pointr = head_;
        for (int j = 1; j <= col; ++j) {
            const double a1 = wa[j - 1];
            const double a2 = theta_ * wa[col + j - 1];
            for (int i = 1; i <= nfree_; ++i) {
                const int k = index_[i - 1];
                r_[i - 1] += WY(k, pointr) * a1 + WS(k, pointr) * a2;
            }
            pointr = nxt(pointr);
        }
        return 0;
    }

    // subspace minimisation over the free variables, then the projection /
    // backtracking of L-BFGS-B 3.0; z becomes the end point of the search direction
    int subsm() {
        const int nsub = nfree_, col = col_;
        if (nsub <= 0) return 0;
        double* d = r_.data();
        double* wv = wv_.data();
        int pointr = head_;
        for (int i = 1; i <= col; ++i) {
            double t1 = 0.0, t2 = 0.0;
            for (int j = 1; j <= nsub; ++j) {
                const int k = index_[j - 1];
                t1 += WY(k, pointr) * d[j - 1];
                t2 += WS(k, pointr) * d[j - 1];
            }
            wv[i - 1] = t1;
            wv[col + i - 1] = theta_ * t2;
            pointr = nxt(pointr);
        }
        const int m2 = 2 * m_, col2 = 2 * col;
        if (dtrsl(wn_.data(), m2, col2, wv, 11)) return -1;
        for (int i = 0; i < col; ++i) wv[i] = -wv[i];
        if (dtrsl(wn_.data(), m2, col2, wv, 1)) return -1;
        pointr = head_;
        for (int jy = 1; jy <= col; ++jy) {
            const int js = col + jy;
            for (int i = 1; i <= nsub; ++i) {
                const int k = index_[i - 1];
                d[i - 1] += WY(k, pointr) * wv[jy - 1] / theta_ + WS(k, pointr) * wv[js - 1];
            }
            pointr = nxt(pointr);
        }
        for (int i = 0; i < nsub; ++i) d[i] *= 1.0 / theta_;

        // try the projected Newton point
        int iword = 0;
        xp_ = z_;
        for (int i = 1; i <= nsub; ++i) {
            const int k = index_[i - 1];
            const double dk = d[i - 1];
            double xk = z_[k - 1];
            const int nb = nbd_[k - 1];
            if (nb != 0) {
                if (nb == 1) {
                    z_[k - 1] = std::fmax(l_[k - 1], xk + dk);
                    if (z_[k - 1] == l_[k - 1]) iword = 1;
                } else if (nb == 2) {
                    xk = std::fmax(l_[k - 1], xk + dk);
                    z_[k - 1] = std::fmin(u_[k - 1], xk);
                    if (z_[k - 1] == l_[k - 1] || z_[k - 1] == u_[k - 1]) iword = 1;
                } else if (nb == 3) {
                    z_[k - 1] = std::fmin(u_[k - 1], xk + dk);
                    if (z_[k - 1] == u_[k - 1]) iword = 1;
                }
            } else {
                z_[k - 1] = xk + dk;
            }
        }
        if (iword == 0) return 0;
        double dd_p = 0.0;
        for (int i = 0; i < n_; ++i) dd_p += (z_[i] - x_[i]) * g_[i];
        if (!(dd_p > 0.0)) return 0;
        // positive directional derivative of the projection: the backtracking step
        z_ = xp_;
        double alpha = 1.0, temp1 = alpha;
        int ibd = 0;
        for (int i = 1; i <= nsub; ++i) {
            const int k = index_[i - 1];
            const double dk = d[i - 1];
            const int nb = nbd_[k - 1];
            if (nb != 0) {
                if (dk < 0.0 && nb <= 2) {
                    const double temp2 = l_[k - 1] - z_[k - 1];
                    if (temp2 >= 0.0) temp1 = 0.0;
                    else if (dk * alpha < temp2) temp1 = temp2 / dk;
                } else if (dk > 0.0 && nb >= 2) {
                    const double temp2 = u_[k - 1] - z_[k - 1];
                    if (temp2 <= 0.0) temp1 = 0.0;
                    else if (dk * alpha > temp2) temp1 = temp2 / dk;
                }
                if (temp1 < alpha) { alpha = temp1; ibd = i; }
            }
        }
        if (alpha < 1.0) {
            const double dk = d[ibd - 1];
            const int k = index_[ibd - 1];
            if (dk > 0.0) { z_[k - 1] = u_[k - 1]; d[ibd - 1] = 0.0; }
            else if (dk < 0.0) { z_[k - 1] = l_[k - 1]; d[ibd - 1] = 0.0; }
        }
        for (int i = 1; i <= nsub; ++i) {
            const int k = index_[i - 1];
            z_[k - 1] += alpha * d[i - 1];
        }
        return 0;
    }

    // the newest correction pair into WS, WY and the middle-matrix blocks SS, SY
    void matupd(double rr, double dr) {
        if (iupdat_ <= m_) {
            col_ = iupdat_;
            itail_ = (head_ + iupdat_ - 2) % m_ + 1;
        } else {
            itail_ = itail_ % m_ + 1;
            head_ = head_ % m_ + 1;
        }
        for (int i = 1; i <= n_; ++i) { WS(i, itail_) = d_[i - 1]; WY(i, itail_) = r_[i - 1]; }
        theta_ = rr / dr;
        const int col = col_;
        if (iupdat_ > m_) {
            for (int j = 1; j <= col - 1; ++j) {
                for (int i = 1; i <= j; ++i) SS(i, j) = SS(i + 1, j + 1);
                for (int i = 0; i < col - j; ++i) SY(j + i, j) = SY(j + 1 + i, j + 1);
            }
        }
        int pointr = head_;
        for (int j = 1; j <= col - 1; ++j) {
            double sy = 0.0, ss = 0.0;
            for (int i = 1; i <= n_; ++i) sy += d_[i - 1] * WY(i, pointr);
            for (int i = 1; i <= n_; ++i) ss += WS(i, pointr) * d_[i - 1];
            SY(col, j) = sy;
            SS(j, col) = ss;
            pointr = nxt(pointr);
        }
        SS(col, col) = stp_ == 1.0 ? dtd_ : stp_ * stp_ * dtd_;
        SY(col, col) = dr;
    }

    // T = theta S'S + L D^-1 L' and its Cholesky factor J' (upper triangle of WT)
    int formt() {
        const int col = col_;
        for (int j = 1; j <= col; ++j) WT(1, j) = theta_ * SS(1, j);
        for (int i = 2; i <= col; ++i) {
            for (int j = i; j <= col; ++j) {
                const int k1 = std::min(i, j) - 1;
                double ddum = 0.0;
                for (int k = 1; k <= k1; ++k) ddum += SY(i, k) * SY(j, k) / SY(k, k);
                WT(i, j) = ddum + theta_ * SS(i, j);
            }
        }
        return dpofa(wt_.data(), m_, col) ? -3 : 0;
    }

    // label 222 of the published driver: Cauchy point, subspace step, line search start
    bool iterate() {
        for (;;) {
            if (!cnstnd_ && col_ > 0) {
                z_ = x_;
                wrk_ = updatd_;
                nseg_ = 0;
            } else {
                if (cauchy() != 0) {
                    reset_memory();
                    continue;
                }
                freev();
                nact_ = n_ - nfree_;
            }
            if (nfree_ != 0 && col_ != 0) {
                int info = 0;
                if (wrk_) info = formk();
                if (info == 0) info = cmprlb();
                if (info == 0) info = subsm();
                if (info != 0) {
                    reset_memory();
                    continue;
                }
            }
            for (int i = 0; i < n_; ++i) d_[i] = z_[i] - x_[i];
            return linesearch(true);
        }
    }

    // lnsrlb and what the driver does with its outcome (labels 666 / 777 / 888)
    bool linesearch(bool first) {
        for (;;) {
            info_ = 0;
            bool new_x = false;
            if (first) {
                dtd_ = ddot(n_, d_.data(), d_.data());
                dnorm_ = std::sqrt(dtd_);
                stpmx_ = 1e10;
                if (cnstnd_) {
                    if (iter_ == 0) {
                        stpmx_ = 1.0;
                    } else {
                        for (int i = 0; i < n_; ++i) {
                            const double a1 = d_[i];
                            if (nbd_[i] != 0) {
                                if (a1 < 0.0 && nbd_[i] <= 2) {
                                    const double a2 = l_[i] - x_[i];
                                    if (a2 >= 0.0) stpmx_ = 0.0;
                                    else if (a1 * stpmx_ < a2) stpmx_ = a2 / a1;
                                } else if (a1 > 0.0 && nbd_[i] >= 2) {
                                    const double a2 = u_[i] - x_[i];
                                    if (a2 <= 0.0) stpmx_ = 0.0;
                                    else if (a1 * stpmx_ > a2) stpmx_ = a2 / a1;
                                }
                            }
                        }
                    }
                }
                stp_ = (iter_ == 0 && !boxed_) ? std::fmin(1.0 / dnorm_, stpmx_) : 1.0;
                t_ = x_;
                r_ = g_;
                fold_ = f_;
                ifun_ = 0;
                iback_ = 0;
                ls_.task = Dcsrch::START;
            }
            first = false;
            gd_ = ddot(n_, g_.data(), d_.data());
            bool fg = false;
            if (ifun_ == 0) {
                gdold_ = gd_;
                if (gd_ >= 0.0) info_ = -4;      // not a descent direction
            }
            if (info_ == 0) {
                ls_.step(f_, gd_, stp_, 1e-3, 0.9, 0.1, 0.0, stpmx_);
                if (ls_.task != Dcsrch::CONV && ls_.task != Dcsrch::WARN) {
                    fg = true;
                    ++ifun_;
                    iback_ = ifun_ - 1;
                    if (stp_ == 1.0) x_ = z_;
                    else for (int i = 0; i < n_; ++i) x_[i] = stp_ * d_[i] + t_[i];
                } else {
                    new_x = true;
                }
            }
            if (info_ != 0 || iback_ >= maxls_) {
                // back to the previous iterate
                x_ = t_;
                g_ = r_;
                f_ = fold_;
                if (col_ == 0) {
                    ++iter_;
                    return finish(kAbnormal);
                }
                reset_memory();            // RESTART_FROM_LNSRCH
                return iterate();
            }
            if (fg) {
                phase_ = kPhaseLnsrch;
                return true;
            }
            (void)new_x;
            // NEW_X
            ++iter_;
            sbgnrm_ = projgr();
            ++nit_;                                  // scipy's driver
            if (nit_ >= maxiter_) return finish(kStopMaxiter);
            if (nfev_ > maxfun_) return finish(kStopMaxfun);
            if (sbgnrm_ <= pgtol_) return finish(kConvPgtol);
            const double ddum = std::fmax(std::fmax(std::fabs(fold_), std::fabs(f_)), 1.0);
            if (fold_ - f_ <= tol_ * ddum) return finish(kConvFactr);
            for (int i = 0; i < n_; ++i) r_[i] = g_[i] - r_[i];
            const double rr = ddot(n_, r_.data(), r_.data());
            double dr, dd;
            if (stp_ == 1.0) {
                dr = gd_ - gdold_;
                dd = -gdold_;
            } else {
                dr = (gd_ - gdold_) * stp_;
                for (int i = 0; i < n_; ++i) d_[i] *= stp_;
                dd = -gdold_ * stp_;
            }
            if (dr <= epsmch_ * dd) {
                updatd_ = false;                     // skip the update
            } else {
                updatd_ = true;
                ++iupdat_;
                matupd(rr, dr);
                if (formt() != 0) reset_memory();
            }
            return iterate();
        }
    }

    int n_, m_, maxls_, maxiter_, maxfun_;
    const double *l_, *u_;
    const int* nbd_;
    double pgtol_, tol_, epsmch_;
    std::vector<double> x_, g_, z_, r_, d_, t_, xp_, ws_, wy_, sy_, ss_, wt_, wn_, wa_, wv_;
    std::vector<int> index_, iwhere_, indx2_;
    double f_ = 0.0, fold_ = 0.0, theta_ = 1.0, gd_ = 0.0, gdold_ = 0.0, stp_ = 0.0, stpmx_ = 0.0, dtd_ = 0.0,
           dnorm_ = 0.0, sbgnrm_ = 0.0;
    int col_ = 0, head_ = 1, itail_ = 0, iupdat_ = 0, iter_ = 0, nseg_ = 0, nfree_ = 0, nact_ = 0, ileave_ = 0,
        nenter_ = 0, ifun_ = 0, iback_ = 0, info_ = 0, nit_ = 0, nfev_ = 0;
    bool updatd_ = false, cnstnd_ = false, boxed_ = true, wrk_ = false;
    Phase phase_ = kPhaseStart;
    int status_ = kRunning;
    Dcsrch ls_;
};

struct Options {
    double ftol, gtol;
    int maxiter, maxfun, maxcor, maxls;
};

// Independent runs from x0 [nruns][nvar] within bounds [nvar][2]; every round
// evaluates the point each live run needs in one fg(batch, X, ids, f, g) call.
// Outputs: x_out [nruns][nvar], f_out [nruns] (the last value delivered to the run,
// scipy's OptimizeResult.fun), stats [nruns][4] = (nit, nfev, status, 0).
template <class FG>
int drive(int nvar, int nruns, const double* x0, const double* bounds, const Options& o, FG&& fg, double* x_out,
          double* f_out, int32_t* stats, int32_t* rounds_out) {
    std::vector<double> lo(nvar), hi(nvar);
    std::vector<int> nbd(nvar, 2);
    for (int i = 0; i < nvar; ++i) { lo[i] = bounds[2 * i]; hi[i] = bounds[2 * i + 1]; }
    const double factr = o.ftol / 2.220446049250313e-16;
    std::vector<Lbfgsb> runs;
    runs.reserve(nruns);
    std::vector<double> xs(nvar);
    for (int r = 0; r < nruns; ++r) {
        runs.emplace_back(nvar, lo.data(), hi.data(), nbd.data(), factr, o.gtol, o.maxcor, o.maxls, o.maxiter, o.maxfun);
        for (int i = 0; i < nvar; ++i) xs[i] = std::min(std::max(x0[(size_t)r * nvar + i], lo[i]), hi[i]);
        runs.back().start(xs.data());
    }
    std::vector<int32_t> live(nruns), next;
    for (int r = 0; r < nruns; ++r) live[r] = r;
    std::vector<double> X((size_t)nruns * nvar), F(nruns), G((size_t)nruns * nvar), last_f(nruns, 0.0);
    std::vector<double> sf_x((size_t)nruns * nvar), sf_g((size_t)nruns * nvar);
    int rounds = 0;
    while (!live.empty()) {
        const int nl = (int)live.size();
        for (int k = 0; k < nl; ++k) std::copy(runs[live[k]].x(), runs[live[k]].x() + nvar, &X[(size_t)k * nvar]);
        if (int rc = fg(nl, X.data(), live.data(), F.data(), G.data())) return rc;
        ++rounds;
        next.clear();
        for (int k = 0; k < nl; ++k) {
            const int r = live[k];
            Lbfgsb& run = runs[r];
            // ScalarFunction's cache: the point and its values
            double* cx = &sf_x[(size_t)r * nvar];
            double* cg = &sf_g[(size_t)r * nvar];
            std::copy(&X[(size_t)k * nvar], &X[(size_t)(k + 1) * nvar], cx);
            std::copy(&G[(size_t)k * nvar], &G[(size_t)(k + 1) * nvar], cg);
            const double cf = F[k];
            run.count_evaluation();
            last_f[r] = cf;
            bool want = run.deliver(cf, cg);
            while (want && std::equal(run.x(), run.x() + nvar, cx)) {   // the same x again: no evaluation
                last_f[r] = cf;
                want = run.deliver(cf, cg);
            }
            if (want) next.push_back(r);
        }
        live.swap(next);
    }
    for (int r = 0; r < nruns; ++r) {
        std::copy(runs[r].x(), runs[r].x() + nvar, x_out + (size_t)r * nvar);
        f_out[r] = last_f[r];
        if (stats) {
            stats[4 * r] = runs[r].nit();
            stats[4 * r + 1] = runs[r].nfev();
            stats[4 * r + 2] = runs[r].status();
            stats[4 * r + 3] = 0;
        }
    }
    if (rounds_out) *rounds_out = rounds;
    return MPO_OK;
}

bool options_ok(int nvar, int nruns, const double* x0, const double* bounds, const MpoLbfgsbOptions* o) {
    if (nvar <= 0 || nruns <= 0 || !x0 || !bounds || !o) return false;
    if (o->maxcor <= 0 || o->maxls <= 0 || o->maxiter <= 0 || o->maxfun <= 0 || !(o->ftol >= 0.0) || !(o->gtol >= 0.0))
        return false;
    for (int i = 0; i < nvar; ++i)
        if (!(bounds[2 * i] <= bounds[2 * i + 1])) return false;
    return true;
}

Options to_options(const MpoLbfgsbOptions* o) {
    return Options{o->ftol, o->gtol, o->maxiter, o->maxfun, o->maxcor, o->maxls};
}

// Rendezvous of the concurrent refits on one device (the cl_min chains' worker
// threads).  A fit registers for its duration; each of its rounds is queued, and
// the first thread that finds every registered fit either queued or already in a
// launched group -- or whose wait reached the window -- launches all queued rounds
// as ONE grouped split sweep on its own stream (mpo::lml_launch_rounds),
// synchronises, and wakes the others; several groups may be in flight on their
// leaders' streams.  A lone fit leads at once.  The grouping changes no result (each theta's arithmetic is its
// own, gp_fit.hip LmlGroup); it divides the launches per round of all chains by
// their number -- the one-GPU bound of concurrent refits (r05: ~115k small kernels/s
// over 8 chains, ~6 per round, profiles/r05/).
struct LmlBatcher {
    int device = -1;
    std::chrono::microseconds window{40};
    std::mutex mu;
    std::condition_variable cv;
    int active = 0;      // registered fits
    int inflight = 0;    // rounds in launched groups, not yet done
    struct Req {
        mpo::LmlRound round;
        bool taken = false, done = false;
        int rc = 0;
        std::string err;
    };
    std::vector<Req*> pend;
    long long launches = 0, rounds = 0;

    void enter() {
        std::lock_guard<std::mutex> lk(mu);
        ++active;
    }
    void leave() {
        std::lock_guard<std::mutex> lk(mu);
        --active;
        cv.notify_all();     // a waiting leader may now have every registered fit
    }

    int run(Req& q, hipStream_t s) {
        std::unique_lock<std::mutex> lk(mu);
        pend.push_back(&q);
        cv.notify_all();
        const auto deadline = std::chrono::steady_clock::now() + window;
        for (;;) {
            if (q.done) {
                if (q.rc != MPO_OK) mpo::set_error("%s", q.err.c_str());
                return q.rc;
            }
            if (q.taken) {
                cv.wait(lk);
                continue;
            }
            if ((int)pend.size() >= active - inflight || std::chrono::steady_clock::now() >= deadline) {
                std::vector<Req*> mine;
                mine.swap(pend);
                for (Req* m : mine) m->taken = true;
                inflight += (int)mine.size();
                lk.unlock();
                // one launch set per dimension d present (a process may run searches over
                // different spaces on one GPU), in queue order
                std::vector<mpo::LmlRound> rs;
                rs.reserve(mine.size());
                std::vector<bool> used(mine.size(), false);
                int rc = MPO_OK;
                long long sets = 0;
                for (size_t i = 0; i < mine.size() && rc == MPO_OK; ++i) {
                    if (used[i]) continue;
                    rs.clear();
                    for (size_t j = i; j < mine.size(); ++j)
                        if (!used[j] && mine[j]->round.d == mine[i]->round.d) {
                            rs.push_back(mine[j]->round);
                            used[j] = true;
                        }
                    rc = mpo::lml_launch_rounds(rs.data(), (int)rs.size(), s);
                    ++sets;   // one launch set per distinct d
                }
                if (rc == MPO_OK) {
                    const hipError_t e = hipStreamSynchronize(s);
                    if (e != hipSuccess) {
                        mpo::set_error("lml batcher: hipStreamSynchronize: %s", hipGetErrorString(e));
                        rc = MPO_EHIP;
                    }
                }
                const std::string err = rc != MPO_OK ? std::string(mpo_last_error()) : std::string();
                lk.lock();
                inflight -= (int)mine.size();
                launches += sets;
                rounds += (long long)mine.size();
                for (Req* m : mine) {
                    m->rc = rc;
                    m->err = err;
                    m->done = true;
                }
                cv.notify_all();
                continue;
            }
            cv.wait_until(lk, deadline);
        }
    }
};

}  // namespace

extern "C" {

int mpo_gp_lml_batcher_create(int device, void** handle) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && device >= 0, "mpo_gp_lml_batcher_create: bad arguments");
    auto* b = new LmlBatcher();
    b->device = device;
    *handle = b;
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_gp_lml_batcher_destroy(void* handle) {
    MPO_GUARD_BEGIN
    delete static_cast<LmlBatcher*>(handle);
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_gp_lml_batcher_stats(const void* handle, int64_t* launches, int64_t* rounds) {
    MPO_CHECK_ARG(handle && launches && rounds, "mpo_gp_lml_batcher_stats: null pointer");
    auto* b = const_cast<LmlBatcher*>(static_cast<const LmlBatcher*>(handle));
    std::lock_guard<std::mutex> lk(b->mu);
    *launches = b->launches;
    *rounds = b->rounds;
    return MPO_OK;
}

int mpo_lbfgsb_batched(int nvar, int nruns, const double* x0, const double* bounds, const MpoLbfgsbOptions* opts,
                       mpo_fg_batch_fn fg, void* user, double* x_out, double* f_out, int32_t* stats,
                       int32_t* rounds) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(options_ok(nvar, nruns, x0, bounds, opts) && fg && x_out && f_out,
                  "mpo_lbfgsb_batched: bad arguments (nvar=%d nruns=%d)", nvar, nruns);
    auto eval = [&](int b, const double* X, const int32_t* ids, double* f, double* g) -> int {
        const int rc = fg(b, X, ids, f, g, user);
        if (rc != 0) mpo::set_error("mpo_lbfgsb_batched: objective callback returned %d", rc);
        return rc != 0 ? MPO_EINVAL : 0;
    };
    return drive(nvar, nruns, x0, bounds, to_options(opts), eval, x_out, f_out, stats, rounds);
    MPO_GUARD_END
}

int mpo_gp_fit_lml_host(const double* X, const double* y_norm, int n, int d, const double* starts, int nruns,
                        const double* bounds, const MpoLbfgsbOptions* opts, double* theta_host, double* out_host,
                        void* dev_io, size_t io_bytes, void* ws, size_t ws_bytes, double* x_out, double* f_out,
                        int32_t* stats, int32_t* rounds, void* batcher, void* stream) {
    MPO_GUARD_BEGIN
    const int k = d + 2;
    MPO_CHECK_ARG(X && y_norm && theta_host && out_host && x_out && f_out && n > 0 && d > 0,
                  "mpo_gp_fit_lml_host: bad arguments");
    MPO_CHECK_ARG(options_ok(k, nruns, starts, bounds, opts), "mpo_gp_fit_lml_host: bad options / bounds");
    MPO_CHECK_ARG(io_bytes >= mpo_gp_lml_io_bytes(d, nruns), "mpo_gp_fit_lml_host: io buffer too small");
    MPO_CHECK_ARG(ws_bytes >= mpo_gp_lml_ws_bytes(n, d, nruns), "mpo_gp_fit_lml_host: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    mpo::StreamDeviceScope on_device(s);
    // grouped rounds through the batcher: the fused split sweep, pinned theta / out
    // buffers (their device views), a batcher of this stream's device
    LmlBatcher* bt = static_cast<LmlBatcher*>(batcher);
    mpo::LmlRound base{};
    if (bt) {
        int dev = -1;
        hipPointerAttribute_t ta{}, oa{};
        const bool ok = hipStreamGetDevice(s, &dev) == hipSuccess && dev == bt->device && mpo::lml_groupable(n, d) &&
                        hipPointerGetAttributes(&ta, theta_host) == hipSuccess && ta.type == hipMemoryTypeHost &&
                        ta.devicePointer && hipPointerGetAttributes(&oa, out_host) == hipSuccess &&
                        oa.type == hipMemoryTypeHost && oa.devicePointer;
        if (!ok) {
            (void)hipGetLastError();
            bt = nullptr;
        } else {
            base.X = X;
            base.y = y_norm;
            base.n = n;
            base.d = d;
            base.theta_dev = static_cast<double*>(dev_io);
            base.theta_src = static_cast<const double*>(ta.devicePointer);
            base.out = static_cast<double*>(oa.devicePointer);
            base.ws = reinterpret_cast<double*>(mpo::align_up(reinterpret_cast<uintptr_t>(ws), 256));
        }
    }
    struct Registration {
        LmlBatcher* b;
        explicit Registration(LmlBatcher* b_) : b(b_) { if (b) b->enter(); }
        ~Registration() { if (b) b->leave(); }
    } reg(bt);
    // one round: theta (pinned) -> lml | grad | info (pinned); the objective is -lml, -grad
    auto eval = [&](int b, const double* T, const int32_t*, double* f, double* g) -> int {
        std::memcpy(theta_host, T, sizeof(double) * (size_t)b * k);
        int rc;
        if (bt) {
            LmlBatcher::Req q;
            q.round = base;
            q.round.batch = b;
            rc = bt->run(q, s);
        } else {
            rc = mpo_gp_lml_grad_host(X, y_norm, n, d, theta_host, b, out_host, dev_io, io_bytes, ws, ws_bytes,
                                      stream);
        }
        if (rc != MPO_OK) return rc;
        for (int i = 0; i < b; ++i) f[i] = -out_host[i];
        for (size_t i = 0; i < (size_t)b * k; ++i) g[i] = -out_host[b + i];
        return 0;
    };
    return drive(k, nruns, starts, bounds, to_options(opts), eval, x_out, f_out, stats, rounds);
    MPO_GUARD_END
}

int mpo_gp_polish_host(const MpoGpModel* model, const double* starts, const int32_t* acq, int nruns,
                       const double* bounds, const MpoLbfgsbOptions* opts, double y_opt, double xi, double kappa,
                       double* x_host, int32_t* acq_host, double* f_host, double* g_host, double* x_out,
                       double* f_out, int32_t* stats, int32_t* rounds, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(model && acq && x_host && acq_host && f_host && g_host && x_out && f_out,
                  "mpo_gp_polish_host: null pointer");
    const int d = model->d;
    MPO_CHECK_ARG(options_ok(d, nruns, starts, bounds, opts), "mpo_gp_polish_host: bad options / bounds");
    auto eval = [&](int b, const double* Xp, const int32_t* ids, double* f, double* g) -> int {
        std::memcpy(x_host, Xp, sizeof(double) * (size_t)b * d);
        for (int i = 0; i < b; ++i) acq_host[i] = acq[ids[i]];
        const int rc = mpo_gp_acq_grad_host(model, x_host, b, acq_host, y_opt, xi, kappa, f_host, g_host, stream);
        if (rc != MPO_OK) return rc;
        std::memcpy(f, f_host, sizeof(double) * b);
        std::memcpy(g, g_host, sizeof(double) * (size_t)b * d);
        return 0;
    };
    return drive(d, nruns, starts, bounds, to_options(opts), eval, x_out, f_out, stats, rounds);
    MPO_GUARD_END
}

}  // extern "C"
