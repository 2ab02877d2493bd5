"""The subset of h5py that Dorknet's checkpoints use, over the HDF5 C library (ctypes).

The reference saves and loads checkpoints with h5py (network/feed_forward_network.py:90-139
and each layer's save_to_h5 / load_from_h5, e.g. layers/convolution.py:226-281).  h5py is
not installed in this image, but the HDF5 C library is (libhdf5 1.10, e.g. from the conda
tree), so this module binds the calls those checkpoints need and writes the objects h5py
writes for the same Python values:

=====================================  ===========================================
value assigned (h5py)                  HDF5 object written (same as h5py 3.x)
=====================================  ===========================================
``create_dataset(name, dtype=f4)``     dataset with a null dataspace (``h5py.Empty``)
``create_dataset(name, shape, dtype)`` contiguous little-endian dataset; ``d[:] = a``
``attrs[k] = "str"``                   scalar variable-length UTF-8 string
``attrs[k] = ["a", "b"]``              1-D array of variable-length UTF-8 strings
``attrs[k] = np.string_("l2")``        scalar fixed-length ASCII string (NULLPAD)
``attrs[k] = True``                    scalar enum {FALSE = 0, TRUE = 1} over int8
``attrs[k] = 3`` / ``0.95``            scalar int64 / float64
=====================================  ===========================================

Reading returns what h5py returns: ``str`` for variable-length strings, ``numpy.bytes_`` for
fixed-length ones, an object array of ``str`` for string arrays, ``numpy.bool_`` for the
boolean enum, numpy scalars for numbers and ``ds[:]`` / ``ds[()]`` as numpy arrays.

This is checkpoint I/O, not part of the GPU hot path; ``File`` raises ``ImportError`` when
no HDF5 library can be found (``DORKNET_LIBHDF5`` names one explicitly).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os

import numpy as np

hid_t = ctypes.c_int64
herr_t = ctypes.c_int
htri_t = ctypes.c_int
hsize_t = ctypes.c_ulonglong

H5F_ACC_RDONLY, H5F_ACC_RDWR, H5F_ACC_TRUNC, H5F_ACC_EXCL = 0x0, 0x1, 0x2, 0x4
H5P_DEFAULT = 0
H5S_ALL = 0
H5S_SCALAR, H5S_SIMPLE, H5S_NULL = 0, 1, 2
H5T_INTEGER, H5T_FLOAT, H5T_STRING, H5T_ENUM = 0, 1, 3, 8
H5T_VARIABLE = ctypes.c_size_t(-1).value
H5T_CSET_ASCII, H5T_CSET_UTF8 = 0, 1
H5T_STR_NULLTERM, H5T_STR_NULLPAD = 0, 1
H5T_SGN_NONE = 0
H5I_GROUP, H5I_DATASET = 2, 5
H5_INDEX_NAME, H5_ITER_INC = 0, 0

_CANDIDATES = ("/opt/conda/lib/libhdf5.so.103", "/opt/conda/lib/libhdf5.so", "libhdf5.so.103", "libhdf5.so")

_lib = None


class _H5GInfo(ctypes.Structure):
    _fields_ = [("storage_type", ctypes.c_int), ("nlinks", hsize_t), ("max_corder", ctypes.c_int64),
                ("mounted", ctypes.c_bool)]


def _load():
    global _lib
    if _lib is not None:
        return _lib
    names = [os.environ["DORKNET_LIBHDF5"]] if os.environ.get("DORKNET_LIBHDF5") else []
    found = ctypes.util.find_library("hdf5")
    names += list(_CANDIDATES) + ([found] if found else [])
    err = None
    for n in names:
        try:
            lib = ctypes.CDLL(n)
            break
        except OSError as e:
            err = e
    else:
        raise ImportError("h5 checkpoints need h5py or the HDF5 C library (set DORKNET_LIBHDF5); "
                          "none found: {}".format(err))
    sig = {
        "H5open": (herr_t, []),
        "H5Eset_auto2": (herr_t, [hid_t, ctypes.c_void_p, ctypes.c_void_p]),
        "H5Fcreate": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t, hid_t]),
        "H5Fopen": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t]),
        "H5Fclose": (herr_t, [hid_t]),
        "H5Fflush": (herr_t, [hid_t, ctypes.c_int]),
        "H5Gcreate2": (hid_t, [hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t]),
        "H5Gclose": (herr_t, [hid_t]),
        "H5Gget_info": (herr_t, [hid_t, ctypes.POINTER(_H5GInfo)]),
        "H5Lexists": (htri_t, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Lget_name_by_idx": (ctypes.c_ssize_t, [hid_t, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, hsize_t,
                                                  ctypes.c_char_p, ctypes.c_size_t, hid_t]),
        "H5Oopen": (hid_t, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Oclose": (herr_t, [hid_t]),
        "H5Iget_type": (ctypes.c_int, [hid_t]),
        "H5Pcreate": (hid_t, [hid_t]),
        "H5Pclose": (herr_t, [hid_t]),
        "H5Pset_create_intermediate_group": (herr_t, [hid_t, ctypes.c_uint]),
        "H5Screate": (hid_t, [ctypes.c_int]),
        "H5Screate_simple": (hid_t, [ctypes.c_int, ctypes.POINTER(hsize_t), ctypes.POINTER(hsize_t)]),
        "H5Sclose": (herr_t, [hid_t]),
        "H5Sget_simple_extent_type": (ctypes.c_int, [hid_t]),
        "H5Sget_simple_extent_ndims": (ctypes.c_int, [hid_t]),
        "H5Sget_simple_extent_dims": (ctypes.c_int, [hid_t, ctypes.POINTER(hsize_t), ctypes.POINTER(hsize_t)]),
        "H5Dcreate2": (hid_t, [hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t, hid_t]),
        "H5Dclose": (herr_t, [hid_t]),
        "H5Dget_space": (hid_t, [hid_t]),
        "H5Dget_type": (hid_t, [hid_t]),
        "H5Dwrite": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Dread": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Acreate2": (hid_t, [hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t]),
        "H5Aopen": (hid_t, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Aexists": (htri_t, [hid_t, ctypes.c_char_p]),
        "H5Adelete": (herr_t, [hid_t, ctypes.c_char_p]),
        "H5Aclose": (herr_t, [hid_t]),
        "H5Awrite": (herr_t, [hid_t, hid_t, ctypes.c_void_p]),
        "H5Aread": (herr_t, [hid_t, hid_t, ctypes.c_void_p]),
        "H5Aget_space": (hid_t, [hid_t]),
        "H5Aget_type": (hid_t, [hid_t]),
        "H5Aget_name_by_idx": (ctypes.c_ssize_t, [hid_t, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, hsize_t,
                                                  ctypes.c_char_p, ctypes.c_size_t, hid_t]),
        "H5Aget_num_attrs": (ctypes.c_int, [hid_t]),
        "H5Tcopy": (hid_t, [hid_t]),
        "H5Tclose": (herr_t, [hid_t]),
        "H5Tset_size": (herr_t, [hid_t, ctypes.c_size_t]),
        "H5Tget_size": (ctypes.c_size_t, [hid_t]),
        "H5Tset_cset": (herr_t, [hid_t, ctypes.c_int]),
        "H5Tset_strpad": (herr_t, [hid_t, ctypes.c_int]),
        "H5Tget_class": (ctypes.c_int, [hid_t]),
        "H5Tget_sign": (ctypes.c_int, [hid_t]),
        "H5Tis_variable_str": (htri_t, [hid_t]),
        "H5Tenum_create": (hid_t, [hid_t]),
        "H5Tenum_insert": (herr_t, [hid_t, ctypes.c_char_p, ctypes.c_void_p]),
        "H5Tget_super": (hid_t, [hid_t]),
        "H5Dvlen_reclaim": (herr_t, [hid_t, hid_t, hid_t, ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.H5open() < 0:
        raise ImportError("H5open failed")
    lib.H5Eset_auto2(H5P_DEFAULT, None, None)  # errors come back as return codes, not stderr
    _lib = lib
    return lib


def _g(name):
    return hid_t.in_dll(_load(), name).value


def _check(v, what):
    if v < 0:
        raise OSError("HDF5: {} failed".format(what))
    return v


def _native(dtype):
    """(memory type, file type) for a numeric numpy dtype (little-endian standard file types,
    as h5py writes them)."""
    dt = np.dtype(dtype)
    table = {
        np.dtype(np.float32): ("H5T_NATIVE_FLOAT_g", "H5T_IEEE_F32LE_g"),
        np.dtype(np.float64): ("H5T_NATIVE_DOUBLE_g", "H5T_IEEE_F64LE_g"),
        np.dtype(np.int8): ("H5T_NATIVE_SCHAR_g", "H5T_STD_I8LE_g"),
        np.dtype(np.int16): ("H5T_NATIVE_SHORT_g", "H5T_STD_I16LE_g"),
        np.dtype(np.int32): ("H5T_NATIVE_INT_g", "H5T_STD_I32LE_g"),
        np.dtype(np.int64): ("H5T_NATIVE_LLONG_g", "H5T_STD_I64LE_g"),
        np.dtype(np.uint8): ("H5T_NATIVE_UCHAR_g", "H5T_STD_U8LE_g"),
        np.dtype(np.uint32): ("H5T_NATIVE_UINT_g", "H5T_STD_U32LE_g"),
        np.dtype(np.uint64): ("H5T_NATIVE_ULLONG_g", "H5T_STD_U64LE_g"),
    }
    if dt not in table:
        raise TypeError("unsupported dtype for h5 checkpoints: {}".format(dt))
    m, f = table[dt]
    return _g(m), _g(f)


def _bool_type():
    lib = _load()
    t = _check(lib.H5Tenum_create(_g("H5T_NATIVE_SCHAR_g")), "H5Tenum_create")
    for name, v in ((b"FALSE", 0), (b"TRUE", 1)):
        c = ctypes.c_int8(v)
        lib.H5Tenum_insert(t, name, ctypes.byref(c))
    return t


def _str_type(size, utf8):
    lib = _load()
    t = _check(lib.H5Tcopy(_g("H5T_C_S1_g")), "H5Tcopy")
    lib.H5Tset_size(t, size)
    lib.H5Tset_cset(t, H5T_CSET_UTF8 if utf8 else H5T_CSET_ASCII)
    if size != H5T_VARIABLE:
        lib.H5Tset_strpad(t, H5T_STR_NULLPAD)
    return t


def _space(shape):
    lib = _load()
    if shape is None:
        return _check(lib.H5Screate(H5S_NULL), "H5Screate")
    if len(shape) == 0:
        return _check(lib.H5Screate(H5S_SCALAR), "H5Screate")
    dims = (hsize_t * len(shape))(*shape)
    return _check(lib.H5Screate_simple(len(shape), dims, None), "H5Screate_simple")


def _shape_of(space):
    lib = _load()
    kind = lib.H5Sget_simple_extent_type(space)
    if kind == H5S_NULL:
        return None
    n = lib.H5Sget_simple_extent_ndims(space)
    if n <= 0:
        return ()
    dims = (hsize_t * n)()
    lib.H5Sget_simple_extent_dims(space, dims, None)
    return tuple(int(d) for d in dims)


def _dtype_of(t):
    """numpy dtype (or a string / bool marker) of an HDF5 type."""
    lib = _load()
    cls = lib.H5Tget_class(t)
    size = lib.H5Tget_size(t)
    if cls == H5T_FLOAT:
        return np.dtype("<f%d" % size)
    if cls == H5T_INTEGER:
        return np.dtype(("<u%d" if lib.H5Tget_sign(t) == H5T_SGN_NONE else "<i%d") % size)
    if cls == H5T_ENUM:
        return "bool"
    if cls == H5T_STRING:
        return "vstr" if lib.H5Tis_variable_str(t) > 0 else ("fstr", size)
    raise TypeError("unsupported HDF5 type class {}".format(cls))


class Empty:
    """h5py.Empty: a dataset or attribute with a null dataspace."""

    def __init__(self, dtype):
        self.dtype = np.dtype(dtype)

    def __eq__(self, other):
        return isinstance(other, Empty) and other.dtype == self.dtype

    def __repr__(self):
        return "Empty(dtype={!r})".format(self.dtype)


class AttributeManager:
    def __init__(self, oid):
        self._id = oid

    def __contains__(self, name):
        return _load().H5Aexists(self._id, name.encode()) > 0

    def keys(self):
        lib = _load()
        out = []
        for i in range(lib.H5Aget_num_attrs(self._id)):
            n = lib.H5Aget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, None, 0, H5P_DEFAULT)
            buf = ctypes.create_string_buffer(n + 1)
            lib.H5Aget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, n + 1, H5P_DEFAULT)
            out.append(buf.value.decode())
        return out

    def __iter__(self):
        return iter(self.keys())

    def get(self, name, default=None):
        return self[name] if name in self else default

    def __setitem__(self, name, value):
        lib = _load()
        key = name.encode()
        if lib.H5Aexists(self._id, key) > 0:
            lib.H5Adelete(self._id, key)
        keep = []  # ctypes / numpy buffers that must outlive H5Awrite
        owned = []  # HDF5 types to close
        if isinstance(value, (bool, np.bool_)):
            ftype = mtype = _bool_type()
            owned.append(ftype)
            space = _space(())
            c = ctypes.c_int8(int(bool(value)))
            keep.append(c)
            ptr = ctypes.cast(ctypes.pointer(c), ctypes.c_void_p)
        elif isinstance(value, str):
            ftype = mtype = _str_type(H5T_VARIABLE, True)
            owned.append(ftype)
            space = _space(())
            s = ctypes.c_char_p(value.encode("utf-8"))
            keep.append(s)
            ptr = ctypes.cast(ctypes.pointer(s), ctypes.c_void_p)  # char**
        elif isinstance(value, (bytes, np.bytes_)):
            raw = bytes(value)
            ftype = mtype = _str_type(max(1, len(raw)), False)
            owned.append(ftype)
            space = _space(())
            b = ctypes.create_string_buffer(raw, max(1, len(raw)))
            keep.append(b)
            ptr = ctypes.cast(b, ctypes.c_void_p)
        elif isinstance(value, (list, tuple)) and all(isinstance(v, str) for v in value):
            ftype = mtype = _str_type(H5T_VARIABLE, True)
            owned.append(ftype)
            space = _space((len(value),))
            arr = (ctypes.c_char_p * max(1, len(value)))(*[v.encode("utf-8") for v in value])
            keep.append(arr)
            ptr = ctypes.cast(arr, ctypes.c_void_p)  # char*[n]
        else:
            a = np.asarray(value)
            if a.dtype.kind == "U" or a.dtype == object:
                return self.__setitem__(name, [str(v) for v in a.ravel()])
            if a.dtype == np.bool_:
                if a.ndim == 0:
                    return self.__setitem__(name, bool(a))
                raise TypeError("boolean array attributes are not supported")
            if a.dtype.kind == "S":
                return self.__setitem__(name, np.bytes_(a.item()))
            mtype, ftype = _native(a.dtype)
            a = np.array(a, order="C", copy=True)  # (ascontiguousarray would make a 0-d value 1-d)
            keep.append(a)
            space = _space(a.shape)
            ptr = a.ctypes.data_as(ctypes.c_void_p)
        try:
            attr = _check(lib.H5Acreate2(self._id, key, ftype, space, H5P_DEFAULT, H5P_DEFAULT), "H5Acreate2")
            try:
                _check(lib.H5Awrite(attr, mtype, ptr), "H5Awrite")
            finally:
                lib.H5Aclose(attr)
        finally:
            lib.H5Sclose(space)
            for t in owned:
                lib.H5Tclose(t)
        del keep

    def __getitem__(self, name):
        lib = _load()
        key = name.encode()
        if lib.H5Aexists(self._id, key) <= 0:
            raise KeyError(name)
        attr = _check(lib.H5Aopen(self._id, key, H5P_DEFAULT), "H5Aopen")
        space = lib.H5Aget_space(attr)
        t = lib.H5Aget_type(attr)
        try:
            shape = _shape_of(space)
            kind = _dtype_of(t)
            if shape is None:
                return Empty(np.float32 if not isinstance(kind, np.dtype) else kind)
            n = int(np.prod(shape)) if shape else 1
            if kind == "vstr":
                mt = _str_type(H5T_VARIABLE, True)
                ptrs = (ctypes.c_char_p * n)()
                _check(lib.H5Aread(attr, mt, ptrs), "H5Aread")
                vals = [p.decode("utf-8") if p is not None else "" for p in ptrs]
                lib.H5Dvlen_reclaim(mt, space, H5P_DEFAULT, ptrs)
                lib.H5Tclose(mt)
                if shape == ():
                    return vals[0]
                return np.array(vals, dtype=object).reshape(shape)
            if isinstance(kind, tuple):  # fixed-length string
                size = kind[1]
                buf = ctypes.create_string_buffer(size * n)
                _check(lib.H5Aread(attr, t, buf), "H5Aread")
                raw = buf.raw
                vals = [np.bytes_(raw[i * size:(i + 1) * size].rstrip(b"\0")) for i in range(n)]
                return vals[0] if shape == () else np.array(vals).reshape(shape)
            if kind == "bool":
                mt = _bool_type()
                out = np.zeros(shape, dtype=np.int8)
                _check(lib.H5Aread(attr, mt, out.ctypes.data_as(ctypes.c_void_p)), "H5Aread")
                lib.H5Tclose(mt)
                out = out.astype(np.bool_)
                return out[()] if shape == () else out
            mt, _ = _native(kind)
            out = np.zeros(shape, dtype=kind)
            _check(lib.H5Aread(attr, mt, out.ctypes.data_as(ctypes.c_void_p)), "H5Aread")
            return out[()] if shape == () else out
        finally:
            lib.H5Tclose(t)
            lib.H5Sclose(space)
            lib.H5Aclose(attr)


class Dataset:
    def __init__(self, oid, name):
        self.id = oid
        self.name = name
        self.attrs = AttributeManager(oid)

    @property
    def shape(self):
        lib = _load()
        sp = lib.H5Dget_space(self.id)
        try:
            return _shape_of(sp)
        finally:
            lib.H5Sclose(sp)

    @property
    def dtype(self):
        lib = _load()
        t = lib.H5Dget_type(self.id)
        try:
            return _dtype_of(t)
        finally:
            lib.H5Tclose(t)

    def _whole(self, key):
        if key is Ellipsis or key == () or (isinstance(key, slice) and key == slice(None)):
            return
        raise NotImplementedError("h5 checkpoints read and write whole datasets only ([:] / [()])")

    def __getitem__(self, key):
        self._whole(key)
        shape, dt = self.shape, self.dtype
        if shape is None:
            return Empty(dt)
        out = np.empty(shape, dtype=dt)
        mt, _ = _native(dt)
        _check(_load().H5Dread(self.id, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.ctypes.data_as(ctypes.c_void_p)),
               "H5Dread")
        return out

    def __setitem__(self, key, value):
        self._whole(key)
        shape, dt = self.shape, self.dtype
        a = np.array(np.broadcast_to(np.asarray(value, dtype=dt), shape), order="C", copy=True)
        mt, _ = _native(dt)
        _check(_load().H5Dwrite(self.id, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, a.ctypes.data_as(ctypes.c_void_p)),
               "H5Dwrite")

    def close(self):
        _load().H5Oclose(self.id)


class Group:
    def __init__(self, oid, name="/", file=None):
        self.id = oid
        self.name = name
        self.file = file
        self.attrs = AttributeManager(oid)
        self._open = []

    def _path(self, name):
        return name.encode()

    def __contains__(self, name):
        lib = _load()
        parts = [p for p in name.split("/") if p]
        for i in range(1, len(parts) + 1):
            if lib.H5Lexists(self.id, "/".join(parts[:i]).encode(), H5P_DEFAULT) <= 0:
                return False
        return True

    def __getitem__(self, name):
        lib = _load()
        if name not in self:
            raise KeyError(name)
        oid = _check(lib.H5Oopen(self.id, self._path(name), H5P_DEFAULT), "H5Oopen")
        kind = lib.H5Iget_type(oid)
        full = (self.name.rstrip("/") + "/" + name.strip("/")) if not name.startswith("/") else name
        if kind == H5I_DATASET:
            obj = Dataset(oid, full)
        elif kind == H5I_GROUP:
            obj = Group(oid, full, self.file)
        else:
            lib.H5Oclose(oid)
            raise TypeError("unsupported HDF5 object at {}".format(name))
        self._track(obj)
        return obj

    def _track(self, obj):
        (self.file or self)._open.append(obj)

    def keys(self):
        lib = _load()
        info = _H5GInfo()
        _check(lib.H5Gget_info(self.id, ctypes.byref(info)), "H5Gget_info")
        out = []
        for i in range(info.nlinks):
            n = lib.H5Lget_name_by_idx(self.id, b".", H5_INDEX_NAME, H5_ITER_INC, i, None, 0, H5P_DEFAULT)
            buf = ctypes.create_string_buffer(n + 1)
            lib.H5Lget_name_by_idx(self.id, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, n + 1, H5P_DEFAULT)
            out.append(buf.value.decode())
        return out

    def __iter__(self):
        return iter(self.keys())

    def _lcpl(self):
        lib = _load()
        p = _check(lib.H5Pcreate(_g("H5P_CLS_LINK_CREATE_ID_g")), "H5Pcreate")
        lib.H5Pset_create_intermediate_group(p, 1)
        return p

    def create_group(self, name):
        lib = _load()
        lcpl = self._lcpl()
        try:
            gid = _check(lib.H5Gcreate2(self.id, self._path(name), lcpl, H5P_DEFAULT, H5P_DEFAULT),
                         "H5Gcreate2({})".format(name))
        finally:
            lib.H5Pclose(lcpl)
        g = Group(gid, name, self.file)
        self._track(g)
        return g

    def require_group(self, name):
        return self[name] if name in self else self.create_group(name)

    def create_dataset(self, name, shape=None, dtype=None, data=None):
        lib = _load()
        if data is not None:
            data = np.asarray(data)
            if dtype is None:
                dtype = data.dtype
            if shape is None:
                shape = data.shape
        if dtype is None:
            dtype = np.float32
        _, ftype = _native(dtype)
        space = _space(None if shape is None else tuple(int(s) for s in shape))
        lcpl = self._lcpl()
        try:
            did = _check(lib.H5Dcreate2(self.id, self._path(name), ftype, space, lcpl, H5P_DEFAULT, H5P_DEFAULT),
                         "H5Dcreate2({})".format(name))
        finally:
            lib.H5Pclose(lcpl)
            lib.H5Sclose(space)
        d = Dataset(did, name)
        self._track(d)
        if data is not None:
            d[:] = data
        return d


class File(Group):
    """h5py.File(name, mode) for modes "r", "r+", "w", "w-"/"x", "a"."""

    def __init__(self, name, mode="r"):
        lib = _load()
        fname = os.fsencode(name)
        if mode == "r":
            fid = lib.H5Fopen(fname, H5F_ACC_RDONLY, H5P_DEFAULT)
        elif mode == "r+":
            fid = lib.H5Fopen(fname, H5F_ACC_RDWR, H5P_DEFAULT)
        elif mode == "w":
            fid = lib.H5Fcreate(fname, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT)
        elif mode in ("w-", "x"):
            fid = lib.H5Fcreate(fname, H5F_ACC_EXCL, H5P_DEFAULT, H5P_DEFAULT)
        elif mode == "a":
            fid = (lib.H5Fopen(fname, H5F_ACC_RDWR, H5P_DEFAULT) if os.path.exists(name)
                   else lib.H5Fcreate(fname, H5F_ACC_EXCL, H5P_DEFAULT, H5P_DEFAULT))
        else:
            raise ValueError("invalid mode {!r}".format(mode))
        if fid < 0:
            raise OSError("unable to open {} (mode {!r})".format(name, mode))
        super().__init__(fid, "/", None)
        self.filename = str(name)
        self.mode = mode

    def close(self):
        if self.id is None:
            return
        lib = _load()
        for obj in reversed(self._open):
            if isinstance(obj, Dataset):
                lib.H5Oclose(obj.id)
            else:
                lib.H5Gclose(obj.id)
        self._open = []
        lib.H5Fclose(self.id)
        self.id = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
