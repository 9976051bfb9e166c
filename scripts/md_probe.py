"""MFMA-distance experiment: sd / mu error of the scoring kernel against the golden
fixtures' exact posterior with the direct differences (MPO_GP_DIST=0) and with the
expanded distance forced (MPO_GP_DIST=2, bypassing mpo_gp_prepare's bound), then an
in-process timing A/B at BASELINE configs[1]."""
import glob, os, sys, time
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import synthetic  # noqa: E402
from mpi_opt_amd.gp import DeviceGP  # noqa: E402

for path in sorted(glob.glob("tests/golden/gp_ei_*.npz")):
    z = np.load(path, allow_pickle=False)
    f = {k: z[k] for k in z.files}
    for mode in ("0", "2"):
        os.environ["MPO_GP_DIST"] = mode
        g = DeviceGP(f["X"], f["y"], float(f["amp"]), f["ls"], float(f["noise"]))
        out = g.score(torch.from_numpy(f["C"]).cuda(), float(f["y_opt"]), acqs=("EI",), k=5)
        sd = out["sd"].cpu().numpy()
        mu = out["mu"].cpu().numpy()
        idx = out["topk"]["EI"][0].cpu().numpy()
        print("%-22s dist=%s  max rel sd err %.2e  max abs mu err %.2e  top5 %s  xb %s" % (
            os.path.basename(path), mode, np.max(np.abs(sd - f["sd_exact"]) / f["sd_exact"]),
            np.max(np.abs(mu - f["mu_exact"])), idx.tolist(), bool(g.model.xb)), flush=True)

X, y = synthetic.gp_problem(200, 10, 0)
ls = np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94])
cand = torch.from_numpy(synthetic.gp_candidates(1_000_000, 10, seed=1)).cuda()
gs = {}
for mode in ("0", "2"):
    os.environ["MPO_GP_DIST"] = mode
    gs[mode] = DeviceGP(X, y, 17.4955, ls, 0.0465)
res = {m: [] for m in gs}
for rnd in range(6):
    for mode, g in gs.items():
        os.environ["MPO_GP_DIST"] = mode
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.score(cand, float(np.min(y)), acqs=("EI",), k=5)
        torch.cuda.synchronize()
        if rnd:
            res[mode].append((time.perf_counter() - t0) / 5 * 1e3)
for mode, g in gs.items():
    m = g.model
    if m.xb:
        off = m.xb + (m.np16 + 32) * m.dp * 8 - g._ws.data_ptr()
        flag = float(g._ws[off:off + 8].cpu().numpy().view(np.float64)[0])
        xbo = m.xb - g._ws.data_ptr()
        mqo = xbo + (((m.np16 + 32) * m.dp + 8) * 8 + 255) // 256 * 256
        mq = g._ws[mqo:mqo + 4 * 200 * 8].cpu().numpy().view(np.float64).reshape(2, 200, 2)
        print("direct q[:4]", mq[0, :4, 1], "md q[:4]", mq[1, :4, 1], "mu", mq[0, :4, 0], mq[1, :4, 0])
        bad = np.nonzero(np.abs(mq[1, :, 1] - mq[0, :, 1]) > 1e-9)[0]
        print("bad rows", bad[:20], len(bad))
        dq = np.abs(mq[1, :, 1] - mq[0, :, 1]) / np.maximum(17.4955 - mq[0, :, 1], 1e-300)
        dmu = np.abs(mq[1, :, 0] - mq[0, :, 0]) / (np.abs(mq[0, :, 0]) + 1e-3)
        print("dist=%s flag %.1f  self-check max dq/sd2 %.2e  max dmu %.2e  min sd2 %.3e" % (
            mode, flag, dq.max(), dmu.max(), (17.4955 - mq[0, :, 1]).min()), flush=True)
for mode, v in res.items():
    print("dist=%s median %.3f ms min %.3f ms" % (mode, np.median(v), np.min(v)), flush=True)
