"""Minimal HDF5 reader for the reference's on-disk training data.

The reference trains from HDF5 files: mpi_learn's ``H5Data(features_name=
'features', labels_name='labels')`` over ``glob('.../mnist/*.h5')``, the first
70 % of the files for training and the rest for validation
(/root/reference/hyperparameter_search_option3.py:134-142, 253-259).  h5py is not
part of this image, so this module reads the file format directly (HDF5 format
spec 3.0, numpy only) -- enough for the numeric datasets h5py writes:

* superblock v0/v1 (h5py ``libver='earliest'``, the default) and v2/v3
  (``libver='latest'``);
* object headers v1 and v2 with continuation blocks; groups as symbol tables
  (B-tree v1 + local heap) or compact link messages;
* datatypes: fixed-point and IEEE floating point, either byte order;
* storage: compact, contiguous, and chunked with the B-tree v1 (layout v3),
  single-chunk, implicit and fixed-array (layout v4) chunk indexes;
* filters: deflate (gzip), shuffle, fletcher32.

Anything else (dense link storage, extensible-array / B-tree v2 chunk indexes,
szip, compound or variable-length types) raises ``NotImplementedError`` naming
it.  Pinned by tests/test_h5.py against files written by h5py 3.3 / HDF5 1.10.6
(tests/golden/make_h5_fixtures.py).
"""
from __future__ import annotations

import glob
import os
import struct
import zlib

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"


class H5Error(ValueError):
    pass


def _u(buf, off, n):
    return int.from_bytes(buf[off:off + n], "little")


class _Reader:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.buf = f.read()
        self.path = path
        base = None
        for cand in (0, 512, 1024, 2048, 4096, 8192):
            if self.buf[cand:cand + 8] == SIGNATURE:
                base = cand
                break
        if base is None:
            raise H5Error(f"{path}: not an HDF5 file")
        b = self.buf
        ver = b[base + 8]
        if ver in (0, 1):
            self.so, self.sl = b[base + 13], b[base + 14]
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = _u(b, p, self.so)
            p += 4 * self.so                      # base, free-space, EOF, driver info
            root_entry = p
            self.root = ("symtab_entry", root_entry)
        elif ver in (2, 3):
            self.so, self.sl = b[base + 9], b[base + 10]
            p = base + 12
            self.base = _u(b, p, self.so)
            p += 3 * self.so                      # base, superblock extension, EOF
            self.root = ("ohdr", self.base + _u(b, p, self.so))
        else:
            raise NotImplementedError(f"{path}: superblock version {ver}")
        self.undef = (1 << (8 * self.so)) - 1

    # -- primitives -------------------------------------------------------------
    def addr(self, off):
        return _u(self.buf, off, self.so)

    def length(self, off):
        return _u(self.buf, off, self.sl)

    def at(self, a):
        """File offset of a stored address (addresses are relative to the base)."""
        return self.base + a

    # -- object headers -------------------------------------------------------------
    def messages(self, oh):
        """[(type, data offset, size)] of the object header at file offset ``oh``."""
        b = self.buf
        out = []
        if b[oh:oh + 4] == b"OHDR":
            flags = b[oh + 5]
            p = oh + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            csize = _u(b, p, 1 << (flags & 3))
            p += 1 << (flags & 3)
            blocks = [(p, p + csize, flags)]
            while blocks:
                start, end, fl = blocks.pop(0)
                q = start
                while q + 4 <= end:
                    mtype, msize, mflags = b[q], _u(b, q + 1, 2), b[q + 3]
                    q += 4 + (2 if fl & 0x04 else 0)
                    if mtype == 0x10:
                        a, ln = self.at(self.addr(q)), self.length(q + self.so)
                        if b[a:a + 4] != b"OCHK":
                            raise H5Error("bad v2 continuation block")
                        blocks.append((a + 4, a + ln - 4, fl))
                    elif mtype != 0:
                        out.append((mtype, q, msize))
                    q += msize
            return out
        if b[oh] != 1:
            raise NotImplementedError(f"object header version {b[oh]}")
        nmsg = _u(b, oh + 2, 2)
        size = _u(b, oh + 8, 4)
        blocks = [(oh + 16, oh + 16 + size)]
        while blocks and len(out) < nmsg:
            start, end = blocks.pop(0)
            q = start
            while q + 8 <= end:
                mtype, msize = _u(b, q, 2), _u(b, q + 2, 2)
                q += 8
                if mtype == 0x10:
                    blocks.append((self.at(self.addr(q)), self.at(self.addr(q)) + self.length(q + self.so)))
                elif mtype != 0:
                    out.append((mtype, q, msize))
                q += msize
        return out

    # -- groups ------------------------------------------------------------------------
    def group_links(self, oh):
        """{name: object header offset} of the group whose header is at ``oh``."""
        links = {}
        for mtype, p, _ in self.messages(oh):
            if mtype == 0x11:      # symbol table: v1 B-tree + local heap
                links.update(self._symtab(self.at(self.addr(p)), self.at(self.addr(p + self.so))))
            elif mtype == 0x06:    # link message (compact storage)
                name, target = self._link(p)
                if target is not None:
                    links[name] = target
            elif mtype == 0x02:    # link info
                if self.addr(p + 2 + (8 if self.buf[p + 1] & 1 else 0)) != self.undef:
                    raise NotImplementedError("dense link storage (fractal heap)")
        return links

    def _link(self, p):
        b = self.buf
        flags = b[p + 1]
        q = p + 2
        ltype = 0
        if flags & 0x08:
            ltype = b[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        nlen_size = 1 << (flags & 3)
        nlen = _u(b, q, nlen_size)
        q += nlen_size
        name = b[q:q + nlen].decode("utf-8")
        q += nlen
        if ltype != 0:
            return name, None      # soft / external links are not followed
        return name, self.at(self.addr(q))

    def _symtab(self, btree, heap):
        b = self.buf
        if b[heap:heap + 4] != b"HEAP":
            raise H5Error("bad local heap")
        data = self.at(self.addr(heap + 8 + 2 * self.sl))
        out = {}

        def walk(node):
            if b[node:node + 4] != b"TREE" or b[node + 4] != 0:
                raise H5Error("bad group B-tree node")
            level, used = b[node + 5], _u(b, node + 6, 2)
            p = node + 8 + 2 * self.so + self.sl         # past key 0
            for _ in range(used):
                child = self.at(self.addr(p))
                p += self.so + self.sl
                if level > 0:
                    walk(child)
                    continue
                if b[child:child + 4] != b"SNOD":
                    raise H5Error("bad symbol table node")
                for e in range(_u(b, child + 6, 2)):
                    ent = child + 8 + e * (2 * self.so + 24)
                    noff = self.addr(ent)
                    end = b.index(b"\0", data + noff)
                    out[b[data + noff:end].decode("utf-8")] = self.at(self.addr(ent + self.so))

        walk(btree)
        return out

    def root_links(self):
        kind, off = self.root
        if kind == "ohdr":
            return self.group_links(off)
        # v0/v1 superblock: root symbol-table entry; its scratch pad caches the
        # B-tree / heap addresses, but the object header has the symbol table too
        return self.group_links(self.at(self.addr(off + self.so)))


class Dataset:
    """One numeric dataset: ``shape``, ``dtype``, ``read()`` -> numpy array."""

    def __init__(self, r: _Reader, oh: int, name: str):
        self.r, self.name = r, name
        self.shape = None
        self.dtype = None
        self.layout = None
        self.filters = []
        for mtype, p, size in r.messages(oh):
            if mtype == 0x01:
                self.shape = self._dataspace(p)
            elif mtype == 0x03:
                self.dtype = self._datatype(p)
            elif mtype == 0x08:
                self.layout = (p, size)
            elif mtype == 0x0B:
                self.filters = self._filters(p)
        if self.shape is None or self.dtype is None or self.layout is None:
            raise H5Error(f"{name}: not a dataset")

    def _dataspace(self, p):
        b, r = self.r.buf, self.r
        ver, nd = b[p], b[p + 1]
        q = p + (8 if ver == 1 else 4)
        return tuple(r.length(q + i * r.sl) for i in range(nd))

    def _datatype(self, p):
        b = self.r.buf
        cls, bits0, size = b[p] & 0x0F, b[p + 1], _u(b, p + 4, 4)
        order = ">" if bits0 & 1 else "<"
        if cls == 0:
            return np.dtype(f"{order}{'i' if bits0 & 0x08 else 'u'}{size}")
        if cls == 1:
            return np.dtype(f"{order}f{size}")
        raise NotImplementedError(f"{self.name}: datatype class {cls}")

    def _filters(self, p):
        b = self.r.buf
        ver, n = b[p], b[p + 1]
        q = p + (8 if ver == 1 else 2)
        out = []
        for _ in range(n):
            fid = _u(b, q, 2)
            q += 2
            nlen = 0
            if ver == 1 or fid >= 256:
                nlen = _u(b, q, 2)
                q += 2
            q += 2                                   # flags
            ncd = _u(b, q, 2)
            q += 2
            if ver == 1:
                q += (nlen + 7) & ~7
            else:
                q += nlen
            cd = [_u(b, q + 4 * i, 4) for i in range(ncd)]
            q += 4 * ncd
            if ver == 1 and ncd % 2:
                q += 4
            out.append((fid, cd))
        return out

    # -- storage ----------------------------------------------------------------------
    def read(self):
        r, b = self.r, self.r.buf
        p, _ = self.layout
        ver, cls = b[p], b[p + 1]
        n = int(np.prod(self.shape)) if self.shape else 1
        nbytes = n * self.dtype.itemsize
        if ver not in (3, 4):
            raise NotImplementedError(f"{self.name}: layout message version {ver}")
        if cls == 0:                                  # compact
            size = _u(b, p + 2, 2)
            raw = b[p + 4:p + 4 + size]
        elif cls == 1:                                # contiguous
            a = r.addr(p + 2)
            raw = bytes(nbytes) if a == r.undef else b[r.at(a):r.at(a) + nbytes]
        elif cls == 2:
            return self._read_chunked(p, ver)
        else:
            raise NotImplementedError(f"{self.name}: layout class {cls}")
        return np.frombuffer(raw, dtype=self.dtype, count=n).reshape(self.shape).astype(self.dtype.newbyteorder("="))

    def _read_chunked(self, p, ver):
        r, b = self.r, self.r.buf
        nd = len(self.shape)
        if ver == 3:
            dims = b[p + 2]
            btree = r.addr(p + 3)
            q = p + 3 + r.so
            chunk = tuple(_u(b, q + 4 * i, 4) for i in range(dims))[:nd]
            chunks = self._btree_chunks(r.at(btree), nd) if btree != r.undef else []
        else:
            flags, dims, enc = b[p + 2], b[p + 3], b[p + 4]
            q = p + 5
            chunk = tuple(_u(b, q + enc * i, enc) for i in range(dims))[:nd]
            q += enc * dims
            itype = b[q]
            q += 1
            chunks = self._v4_chunks(itype, q, flags, chunk)
        out = np.zeros(self.shape, dtype=self.dtype.newbyteorder("="))
        csize = int(np.prod(chunk)) * self.dtype.itemsize
        for offs, addr, size, mask in chunks:
            raw = self._unfilter(b[r.at(addr):r.at(addr) + size], mask)
            blk = np.frombuffer(raw[:csize], dtype=self.dtype).reshape(chunk)
            sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, chunk, self.shape))
            out[sl] = blk[tuple(slice(0, x.stop - x.start) for x in sl)]
        return out

    def _btree_chunks(self, node, nd):
        r, b = self.r, self.r.buf
        if b[node:node + 4] != b"TREE" or b[node + 4] != 1:
            raise H5Error(f"{self.name}: bad chunk B-tree node")
        level, used = b[node + 5], _u(b, node + 6, 2)
        ksize = 8 + 8 * (nd + 1)
        p = node + 8 + 2 * r.so
        out = []
        for _ in range(used):
            size, mask = _u(b, p, 4), _u(b, p + 4, 4)
            offs = tuple(_u(b, p + 8 + 8 * i, 8) for i in range(nd))
            child = r.addr(p + ksize)
            if level > 0:
                out.extend(self._btree_chunks(r.at(child), nd))
            else:
                out.append((offs, child, size, mask))
            p += ksize + r.so
        return out

    def _grid(self, chunk):
        counts = [-(-s // c) for s, c in zip(self.shape, chunk)]
        for lin in range(int(np.prod(counts))):
            idx, rem = [], lin
            for cnt in reversed(counts):
                idx.append(rem % cnt)
                rem //= cnt
            yield tuple(i * c for i, c in zip(reversed(idx), chunk))

    def _v4_chunks(self, itype, q, flags, chunk):
        r, b = self.r, self.r.buf
        csize = int(np.prod(chunk)) * self.dtype.itemsize
        if itype == 1:                                # single chunk
            size, mask = csize, 0
            if flags & 0x02:
                size, mask = r.length(q), _u(b, q + r.sl, 4)
                q += r.sl + 4
            return [((0,) * len(chunk), r.addr(q), size, mask)]
        if itype == 2:                                # implicit: chunks back to back
            a = r.addr(q)
            return [(offs, a + i * csize, csize, 0) for i, offs in enumerate(self._grid(chunk))]
        if itype == 3:                                # fixed array
            hdr = r.at(r.addr(q + 1))
            if b[hdr:hdr + 4] != b"FAHD":
                raise H5Error(f"{self.name}: bad fixed-array header")
            client, esize, pbits = b[hdr + 5], b[hdr + 6], b[hdr + 7]
            nent = r.length(hdr + 8)
            dblk = r.at(r.addr(hdr + 8 + r.sl))
            if nent > (1 << pbits):
                raise NotImplementedError(f"{self.name}: paged fixed-array chunk index")
            if b[dblk:dblk + 4] != b"FADB":
                raise H5Error(f"{self.name}: bad fixed-array data block")
            e = dblk + 6 + r.so
            out = []
            for offs in self._grid(chunk):
                a = r.addr(e)
                if client == 1:
                    w = esize - r.so - 4
                    size, mask = _u(b, e + r.so, w), _u(b, e + r.so + w, 4)
                else:
                    size, mask = csize, 0
                if a != r.undef:
                    out.append((offs, a, size, mask))
                e += esize
            return out
        raise NotImplementedError(f"{self.name}: chunk index type {itype} (extensible array / B-tree v2)")

    def _unfilter(self, raw, mask):
        for i, (fid, cd) in reversed(list(enumerate(self.filters))):
            if mask & (1 << i):
                continue
            if fid == 1:
                raw = zlib.decompress(raw)
            elif fid == 2:
                es = cd[0] if cd else self.dtype.itemsize
                n = len(raw) // es
                raw = np.frombuffer(raw[:n * es], dtype=np.uint8).reshape(es, n).T.tobytes() + raw[n * es:]
            elif fid == 3:
                raw = raw[:-4]
            else:
                raise NotImplementedError(f"{self.name}: filter id {fid}")
        return raw


class H5File:
    """``H5File(path)["features"].read()`` -- read-only access to root datasets."""

    def __init__(self, path):
        self.r = _Reader(path)
        self.links = self.r.root_links()

    def keys(self):
        return list(self.links)

    def __contains__(self, name):
        return name in self.links

    def __getitem__(self, name):
        if name not in self.links:
            raise KeyError(f"{self.r.path}: no dataset {name!r} (has {sorted(self.links)})")
        return Dataset(self.r, self.links[name], name)


def load_xy(paths, features_name="features", labels_name="labels"):
    """Concatenate ``features`` / ``labels`` of the files in order, as the
    population engine consumes them: x float32 [n, H*W*C] (row-major = NHWC
    flattening), integer class labels [n] (one-hot rows are arg-maxed)."""
    xs, ys = [], []
    for p in paths:
        f = H5File(p)
        x = f[features_name].read()
        y = f[labels_name].read()
        if y.ndim == 2:
            y = np.argmax(y, axis=1)
        if x.shape[0] != y.shape[0]:
            raise H5Error(f"{p}: {x.shape[0]} features vs {y.shape[0]} labels")
        xs.append(np.ascontiguousarray(x.reshape(x.shape[0], -1), dtype=np.float32))
        ys.append(y.astype(np.int32))
    return np.concatenate(xs), np.concatenate(ys)


def split_files(data_dir, pattern="*.h5", train_fraction=0.70):
    """option3:134-139: all files, the first 70 % for training, the rest for
    validation (sorted here; the reference uses glob's unsorted order)."""
    files = sorted(glob.glob(os.path.join(data_dir, pattern)))
    if not files:
        raise H5Error(f"no {pattern} files in {data_dir}")
    cut = int(len(files) * train_fraction)
    if cut == 0 or cut == len(files):
        raise H5Error(f"{len(files)} {pattern} file(s) in {data_dir}: the {train_fraction:.0%} file split leaves "
                      f"{cut} for training and {len(files) - cut} for validation; both need at least one")
    return files[:cut], files[cut:]
