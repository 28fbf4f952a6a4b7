"""Dataset text reader: the reference's ModelDataLoader with its
per-item np.loadtxt replaced by libpn2io.so (csrc/io_reader.cpp, include/pn2io.h).

  loadtxt(path, delimiter=",")   np.loadtxt(path, delimiter=...) for these files: same float64
                                 bits (correctly rounded parse), same squeezed shape
  load_many(paths, cols)         a batch of files parsed on a native thread pool
  random_sample(points, number)  /root/reference/data_utils/ModelDataLoader.py:33-46, same
                                 numpy global-RNG draw
  ModelDataLoader(root, args, split)
                                 ModelDataLoader.py:48-91: same file list, same items; adds
                                 load_batch(indices) -> the default-collated batch, files parsed
                                 in parallel and the draws taken in item order

The files are the data_build scripts' np.savetxt(fmt='%6f', delimiter=",") output
(data_build/Cube.py:90-94).  Host code only: importing this module loads no GPU library.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpn2io.so")
ABI_VERSION = 1
_lib = None
_i64 = ctypes.c_int64


class Pn2IoError(ValueError):
    """A libpn2io call failed (unreadable file, non-numeric field, ragged rows): np.loadtxt
    raises ValueError / OSError in these cases."""


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("pn2.data: %s is missing -- run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        L.pn2io_abi_version.restype = ctypes.c_int
        L.pn2io_last_error.restype = ctypes.c_char_p
        L.pn2io_shape.argtypes = [ctypes.c_char_p, ctypes.c_char, ctypes.POINTER(_i64),
                                  ctypes.POINTER(_i64)]
        L.pn2io_read_csv_f64.argtypes = [ctypes.c_char_p, ctypes.c_char, _i64, _i64,
                                         ctypes.c_void_p, ctypes.POINTER(_i64)]
        L.pn2io_read_many_f64.argtypes = [ctypes.POINTER(ctypes.c_char_p), _i64, ctypes.c_char,
                                          _i64, _i64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int]
        for f in ("pn2io_shape", "pn2io_read_csv_f64", "pn2io_read_many_f64"):
            getattr(L, f).restype = ctypes.c_int
        if L.pn2io_abi_version() != ABI_VERSION:
            raise ImportError("pn2.data: libpn2io ABI %d != %d" % (L.pn2io_abi_version(), ABI_VERSION))
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        msg = load().pn2io_last_error().decode(errors="replace")
        if rc == -1:
            raise OSError(msg)
        raise Pn2IoError(msg)


def _delim(d):
    b = d.encode() if isinstance(d, str) else bytes(d)
    if len(b) != 1:
        raise ValueError("pn2.data: the delimiter must be one character")
    return b


def _max_rows(path, cols):
    # a data row takes at least 2*cols bytes ("0,0,0\n")
    return os.path.getsize(path) // (2 * cols) + 1


def _squeeze(a):
    """np.loadtxt(ndmin=0): mono-dimensional axes squeezed."""
    return a.squeeze() if a.ndim == 2 and (a.shape[0] == 1 or a.shape[1] == 1) else a


def loadtxt(path, delimiter=","):
    """float64 array of a delimited text file, as np.loadtxt(path, delimiter=delimiter)."""
    L = load()
    p = os.fsencode(path)
    rows, cols = _i64(), _i64()
    _check(L.pn2io_shape(p, _delim(delimiter), ctypes.byref(rows), ctypes.byref(cols)))
    if rows.value == 0:
        return np.empty((0,), np.float64)
    out = np.empty((rows.value, cols.value), np.float64)
    got = _i64()
    _check(L.pn2io_read_csv_f64(p, _delim(delimiter), cols.value, rows.value,
                                out.ctypes.data, ctypes.byref(got)))
    return _squeeze(out)


def load_many(paths, cols, delimiter=",", threads=0):
    """Parse files on a native thread pool -> list of float64 arrays [rows_i, cols]."""
    n = len(paths)
    if n == 0:
        return []
    mr = max(_max_rows(p, cols) for p in paths)
    out = np.empty((n, mr, cols), np.float64)
    rows = np.zeros(n, np.int64)
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * n)(*enc)
    _check(load().pn2io_read_many_f64(arr, n, _delim(delimiter), cols, mr, out.ctypes.data,
                                      rows.ctypes.data, int(threads)))
    return [out[i, :rows[i]] for i in range(n)]


def random_sample(point_cloud, number=1024):
    """ModelDataLoader.py:33-46: `number` rows without replacement (np.random.choice on the
    global numpy RNG), or the cloud itself when it has <= number rows."""
    N, C = point_cloud.shape
    if N <= number:
        return point_cloud
    sample_idx = np.random.choice(N, number, replace=False)
    return point_cloud[sample_idx]


class ModelDataLoader:
    """Drop-in for /root/reference/data_utils/ModelDataLoader.py:48-91 (a map-style dataset:
    torch.utils.data.DataLoader accepts it as is)."""

    cat = ['cube', 'cuboid', 'cylinder', 'h_structure', 'double_cube', 'double_cylinder',
           'cube_cylinder']

    def __init__(self, root, args, split='train'):
        self.root = root
        self.num_category = args.num_category
        self.classes = dict(zip(self.cat, range(len(self.cat))))
        ids = list(range(1, 8001))
        ids = ids[:6001] if split == 'train' else ids[6001:] if split == 'test' else []
        self.datapath = []
        for item in self.cat:
            for i in ids:
                base = root + item + '/' + item + '_' + '{:0>4d}'.format(i)
                self.datapath.append((item, base + '.txt', base + '_rot.txt', base + '_tran.txt'))

    def __len__(self):
        return len(self.datapath)

    @staticmethod
    def _item(label, points, rot, tran):
        points = random_sample(points)
        rot = np.array(rot, dtype=np.float64)
        sign = np.sign(rot[2])
        rot[2] = np.absolute(rot[2])
        return points, label, rot, tran, sign

    def __getitem__(self, index):
        item, pp, rp, tp = self.datapath[index]
        return self._item(self.classes[item], loadtxt(pp), loadtxt(rp), loadtxt(tp))

    def load_batch(self, indices, threads=0):
        """[self[i] for i in indices] default-collated (torch tensors, as a DataLoader batch
        with num_workers=0 yields it), the 3*len(indices) files parsed in parallel."""
        import torch
        ents = [self.datapath[i] for i in indices]
        pts = load_many([e[1] for e in ents], 3, threads=threads)
        rt = load_many([e[2] for e in ents] + [e[3] for e in ents], 3, threads=threads)
        k = len(ents)
        items = [self._item(self.classes[e[0]], _squeeze(pts[j]), _squeeze(rt[j]),
                            _squeeze(rt[k + j])) for j, e in enumerate(ents)]
        return (torch.from_numpy(np.stack([it[0] for it in items])),
                torch.tensor([it[1] for it in items]),
                torch.from_numpy(np.stack([it[2] for it in items])),
                torch.from_numpy(np.stack([it[3] for it in items])),
                torch.from_numpy(np.stack([it[4] for it in items])))


__all__ = ["loadtxt", "load_many", "random_sample", "ModelDataLoader", "Pn2IoError"]
