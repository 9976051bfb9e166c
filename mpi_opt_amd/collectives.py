"""Fixed-layout tensor collectives for the N-rank search.

The reference exchanges pickled Python objects over MPI p2p: rank 0 ``send``s a
parameter list to every rank of a block and ``irecv``s one float back
(/root/reference/coordinator.py:140-150, process_block.py:54-69, 98-102), and
option3 builds the rank layout with ``Split`` / ``allgather``
(/root/reference/hyperparameter_search_option3.py:172-205).  Here every
per-round exchange is a torch.distributed collective on a plain numeric tensor
-- RCCL over xGMI when the group's backend is ``nccl`` (device tensors), gloo on
CPU tensors otherwise:

* a round header: ``broadcast`` of ``HEADER`` int64 words from rank 0;
* tables: ``broadcast`` of an f64 [rows, cols] array whose shape the header (or
  an earlier broadcast) announced;
* variable-length per-rank rows: ``all_gather`` of each rank's (rows, cols),
  then ``all_gather`` of the rows padded to the largest shape;
* candidate slices: ``scatter`` of equal-height row blocks (the last ones padded).

Parameter points cross as (value, type code) pairs so that a rank rebuilds the
exact Python values rank 0 holds: ints stay ints (a model function's JSON must
see ``int``), floats stay floats (f64 carries them bit for bit).
"""
from __future__ import annotations

import numpy as np

HEADER = 16            # int64 words of a round header
CODE_FLOAT, CODE_INT = 0, 1


_INT_T = (int, np.integer)
_NUM_T = (int, float, np.integer, np.floating)


def _is_int(v):
    return isinstance(v, _INT_T) and not isinstance(v, (bool, np.bool_))


def encode_points(points):
    """[[v, ...], ...] -> (values f64 [n, D], codes f64 [n, D]); ints -> CODE_INT.
    Columns are typed at once when uniform (a search space's points are: Integer
    dimensions give ints, Real ones floats), value by value otherwise."""
    n = len(points)
    d = len(points[0]) if n else 0
    if any(len(p) != d for p in points):
        raise ValueError("encode_points: points of different lengths")
    codes = np.zeros((n, d), dtype=np.float64)
    for j in range(d):
        col = [p[j] for p in points]
        types = set(map(type, col))
        if any(issubclass(t, (bool, np.bool_)) or not issubclass(t, _NUM_T) for t in types):
            bad = next(t for t in types if issubclass(t, (bool, np.bool_)) or not issubclass(t, _NUM_T))
            raise TypeError(f"encode_points: only int / float parameters cross ranks (got {bad.__name__})")
        ints = [issubclass(t, _INT_T) for t in types]
        if all(ints):
            codes[:, j] = CODE_INT
        elif any(ints):
            codes[:, j] = [CODE_INT if _is_int(v) else CODE_FLOAT for v in col]
    vals = np.array(points, dtype=np.float64).reshape(n, d)
    if (codes == CODE_INT).any() and np.abs(vals[codes == CODE_INT]).max(initial=0.0) >= 2.0 ** 53:
        raise ValueError("encode_points: an integer does not fit an f64 exactly")
    return vals, codes


def decode_points(vals, codes):
    vals, codes = np.asarray(vals, dtype=np.float64), np.asarray(codes)
    rows = vals.tolist()
    if not len(rows):
        return rows
    for j in range(vals.shape[1]):
        c = codes[:, j] == CODE_INT
        if c.all():
            for r, v in zip(rows, vals[:, j].astype(np.int64).tolist()):
                r[j] = v
        elif c.any():
            for i in np.nonzero(c)[0]:
                rows[i][j] = int(vals[i, j])
    return rows


class TensorChannel:
    """The collectives of one torch.distributed group, on the backend's device."""

    def __init__(self, dist, group=None):
        import torch

        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = str(dist.get_backend(group)).lower()
        # RCCL ("nccl" on ROCm) moves device tensors; gloo host tensors
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    # ---- broadcasts from rank 0 --------------------------------------------------
    def header(self, words=None):
        """Rank 0 passes up to HEADER ints; every rank gets them (int64 [HEADER])."""
        t = self.torch.zeros(HEADER, dtype=self.torch.int64, device=self.device)
        if self.rank == 0:
            w = [int(v) for v in words]
            if len(w) > HEADER:
                raise ValueError("header: too many words")
            t[:len(w)] = self.torch.tensor(w, dtype=self.torch.int64)
        self.dist.broadcast(t, src=0, group=self.group)
        return [int(v) for v in t.cpu().tolist()]

    def bcast(self, arr, shape, dtype=np.float64):
        """Rank 0's array (others pass None) of the agreed ``shape`` on every rank."""
        tdt = self.torch.float64 if dtype == np.float64 else self.torch.int64
        if self.rank == 0:
            a = np.ascontiguousarray(np.asarray(arr, dtype=dtype).reshape(shape))
            t = self.torch.from_numpy(a).to(self.device)
        else:
            t = self.torch.empty(tuple(shape), dtype=tdt, device=self.device)
        if t.numel():
            self.dist.broadcast(t, src=0, group=self.group)
        return t.cpu().numpy()

    # ---- per-rank rows ---------------------------------------------------------
    def gather_rows(self, rows, dtype=np.float64):
        """Each rank's 2-D array (any height, any width) -> list over ranks (all ranks)."""
        torch = self.torch
        a = np.asarray(rows, dtype=dtype)
        if a.ndim != 2:
            a = a.reshape(len(a), -1) if a.size else np.zeros((0, 0), dtype=dtype)
        shp = torch.tensor(list(a.shape), dtype=torch.int64, device=self.device)
        shapes = [torch.zeros(2, dtype=torch.int64, device=self.device) for _ in range(self.world)]
        self.dist.all_gather(shapes, shp, group=self.group)
        shapes = [tuple(int(v) for v in s.cpu().tolist()) for s in shapes]
        h = max(s[0] for s in shapes)
        w = max(s[1] for s in shapes)
        tdt = torch.float64 if dtype == np.float64 else torch.int64
        if h == 0 or w == 0:
            return [np.zeros(s, dtype=dtype) for s in shapes]
        pad = np.zeros((h, w), dtype=dtype)
        pad[:a.shape[0], :a.shape[1]] = a
        mine = torch.from_numpy(pad).to(self.device)
        outs = [torch.empty((h, w), dtype=tdt, device=self.device) for _ in range(self.world)]
        self.dist.all_gather(outs, mine, group=self.group)
        return [o.cpu().numpy()[:s[0], :s[1]] for o, s in zip(outs, shapes)]

    def gather_text(self, text, width=1024):
        """One short string per rank (an error message, '' for none) -> list over ranks."""
        b = (text or "").encode("utf-8", errors="replace")[:width]
        row = np.zeros((1, width + 1), dtype=np.int64)
        row[0, 0] = len(b)
        row[0, 1:1 + len(b)] = np.frombuffer(b, dtype=np.uint8)
        out = []
        for r in self.gather_rows(row, dtype=np.int64):
            n = int(r[0, 0])
            out.append(bytes(r[0, 1:1 + n].astype(np.uint8)).decode("utf-8", errors="replace"))
        return out

    # ---- candidate slices ------------------------------------------------------
    def scatter_rows(self, full, m, d, as_tensor=False):
        """Rank 0's [m, d] f64 rows split as rank r's [r*m//W, (r+1)*m//W) -> this rank's
        block (numpy, or the received tensor -- on the GPU under RCCL -- with ``as_tensor``)."""
        torch = self.torch
        h = max((r + 1) * m // self.world - r * m // self.world for r in range(self.world))
        out = torch.empty((h, d), dtype=torch.float64, device=self.device)
        parts = None
        if self.rank == 0:
            src = np.ascontiguousarray(np.asarray(full, dtype=np.float64).reshape(m, d))
            parts = []
            for r in range(self.world):
                s0, s1 = r * m // self.world, (r + 1) * m // self.world
                blk = torch.zeros((h, d), dtype=torch.float64, device=self.device)
                if s1 > s0:
                    blk[:s1 - s0] = torch.from_numpy(src[s0:s1]).to(self.device)
                parts.append(blk)
        if self.world == 1:
            out.copy_(parts[0])
        else:
            self.dist.scatter(out, parts, src=0, group=self.group)
        s0, s1 = self.rank * m // self.world, (self.rank + 1) * m // self.world
        if as_tensor:
            return out[:s1 - s0], s0, s1
        return out.cpu().numpy()[:s1 - s0], s0, s1
