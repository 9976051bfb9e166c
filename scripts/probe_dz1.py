import sys, numpy as np, torch
sys.path.insert(0, '.')
from tests.test_train_gpu import dataset, make_engine, oracle_for, orders, BATCH
from oracle import cnn as C
members = [(48,3,2,60,1e-3,0.25,0),(49,3,2,60,1e-3,0.25,1),(50,3,2,60,1e-3,0.25,2),(50,2,2,60,1e-3,0.25,3),(33,3,2,60,1e-3,0.25,4)]
x, y = dataset(1)
eng, specs, init = make_engine(members)
tr, va = orders(members, x)
eng.train_step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), torch.from_numpy(tr).cuda(), 0)
torch.cuda.synchronize()
for i, s in enumerate(specs):
    o = oracle_for(s, init[i])
    _, _, _, c = o.forward(x[tr[i][:BATCH]], y[tr[i][:BATCH]], step=0, train=True)
    # oracle dz2, dz1
    P = o.params; g = o.g
    dh = (c["dz3"] @ P["w4"].T) * c["m2"] * (c["h"] > 0)
    dflat = (dh @ P["w3"].T) * c["m1"]
    da2 = C.maxpool_bwd(dflat.reshape(c["pool_shape"]), c["arg"], c["a2"].shape, g["p"])
    dz2 = da2 * (c["a2"] > 0)
    _, _, da1 = C.conv_bwd(dz2, c["c2"], c["a1"].shape, P["w2"])
    dz1 = da1 * (c["a1"] > 0)
    H1, H2, F = g["H1"], g["H2"], g["F"]
    ddz2 = eng.activation(i, "dz2", (BATCH, H2, H2, F))
    ddz1 = eng.activation(i, "dz1", (BATCH, H1, H1, F))
    w2t = eng.activation(i, "w2t", (s.kernel_size, s.kernel_size, F, F))
    e2 = np.abs(ddz2 - dz2).max() / np.abs(dz2).max()
    e1 = np.abs(ddz1 - dz1)
    print("F=%d k=%d dz2 err %.2e dz1 err %.2e" % (F, s.kernel_size, e2, e1.max() / np.abs(dz1).max()))
    w2 = P["w2"]; k = s.kernel_size
    ref_w2t = w2[::-1, ::-1].transpose(0, 1, 3, 2)
    print("   w2t err", np.abs(w2t - ref_w2t).max())
    if e1.max() / np.abs(dz1).max() > 1e-4:
        bad = np.argwhere(e1 > 1e-4 * np.abs(dz1).max())
        print("   bad count", len(bad), "samples", np.unique(bad[:, 0])[:10], "rows", np.unique(bad[:, 1]), "cols", np.unique(bad[:, 2])[:30], "chans", np.unique(bad[:, 3]))
