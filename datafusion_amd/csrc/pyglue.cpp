/* _dfmi_glue: the Python binding's per-batch FFI marshalling, native.
 *
 * The Python mirror of the relations (datafusion_amd/execution) hands many
 * small host batches to dfmi_filter_project_host_batches per call
 * (csv_sql.rs:49-62 pulls 1024-row batches). Filling the C-ABI structs
 * (dfmi_column per column, dfmi_batch per batch, include/dfmi.h) from the
 * Python Array objects costs ~1 us per column in Python; this module walks
 * the same objects through the CPython API instead. It reads, per Array:
 * data_type, length, null_count, offset (from the instance dict) and the
 * data pointer of its values / validity / offsets tensors -- exactly what
 * engine.column_struct() reads -- and refuses any column whose buffers are
 * not in host memory. Tensors are read through torch's own C++ handle
 * (THPVariable_Unpack: no Python-level is_cpu / data_ptr() calls, ~5 ns
 * instead of ~220 ns per buffer).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#include <torch/csrc/autograd/python_variable.h>

typedef struct {
    int32_t type, reserved;
    int64_t length, null_count;
    uint64_t validity, values, offsets;
    int64_t offset;
} col_rec; /* dfmi_column */

typedef struct {
    int32_t num_columns, reserved;
    int64_t num_rows;
    uint64_t columns;
} batch_rec; /* dfmi_batch */

typedef struct {
    uint64_t values, validity, offsets, data;
    int64_t data_capacity;
    int32_t type, passthrough_column;
    int64_t length, null_count, data_length;
} out_rec; /* dfmi_out_column */

static PyObject *s_columns, *s__columns, *s_data_type, *s_length, *s_null_count, *s_validity, *s_values,
    *s_offsets, *s_offset, *s_schema, *s__blk, *s__vo, *s__vn, *s__bo, *s__bn, *s__oo, *s__on;

/* Integer attribute `name` of `o`: from the instance dict when it is there
 * (a borrowed lookup), else by attribute lookup. */
static int get_i64(PyObject* o, PyObject* name, int64_t* out) {
    PyObject** dp = _PyObject_GetDictPtr(o);
    PyObject* v = dp && *dp ? PyDict_GetItemWithError(*dp, name) : NULL;
    if (v) {
        Py_INCREF(v);
    } else {
        if (PyErr_Occurred()) return -1;
        v = PyObject_GetAttr(o, name);
        if (!v) return -1;
    }
    *out = PyLong_AsLongLong(v);
    Py_DECREF(v);
    return (*out == -1 && PyErr_Occurred()) ? -1 : 0;
}

/* Data pointer of tensor attribute `name` of array `a` (0 for None); fails
 * unless the tensor is in host memory. A BlockArray (arrow.py) whose buffer
 * view was not made yet is read from its block and byte offset (`lazy_off`,
 * e.g. "_vo") without making the view. */
static int get_ptr(PyObject* a, PyObject* name, uint64_t* out, PyObject* lazy_off) {
    PyObject** dp = _PyObject_GetDictPtr(a);
    PyObject* t = dp && *dp ? PyDict_GetItemWithError(*dp, name) : NULL;
    if (!t && !PyErr_Occurred() && dp && *dp) {
        PyObject* blk = PyDict_GetItemWithError(*dp, s__blk);
        PyObject* off = blk ? PyDict_GetItemWithError(*dp, lazy_off) : NULL;
        if (off && THPVariable_Check(blk)) {
            const at::Tensor& x = THPVariable_Unpack(blk);
            if (!x.is_cpu()) {
                PyErr_SetString(PyExc_ValueError, "filter_project_host_batches takes host batches");
                return -1;
            }
            const long long o = PyLong_AsLongLong(off);
            if (o == -1 && PyErr_Occurred()) return -1;
            *out = (uint64_t)(uintptr_t)x.data_ptr() + (uint64_t)o;
            return 0;
        }
    }
    if (t) {
        Py_INCREF(t);
    } else {
        if (PyErr_Occurred()) return -1;
        t = PyObject_GetAttr(a, name);
        if (!t) return -1;
    }
    int rc = 0;
    if (t == Py_None) {
        *out = 0;
    } else if (!THPVariable_Check(t)) {
        PyErr_SetString(PyExc_TypeError, "an Array buffer is not a torch.Tensor");
        rc = -1;
    } else {
        const at::Tensor& x = THPVariable_Unpack(t);
        if (!x.is_cpu()) {
            PyErr_SetString(PyExc_ValueError, "filter_project_host_batches takes host batches");
            rc = -1;
        } else {
            *out = (uint64_t)(uintptr_t)x.data_ptr();
        }
    }
    Py_DECREF(t);
    return rc;
}

/* pack_host_batches(batches, ncols, cols_buf, batches_buf) -> None
 * cols_buf: writable, >= len(batches) * ncols dfmi_column records;
 * batches_buf: writable, >= len(batches) dfmi_batch records. Each batch's
 * `columns` pointer points into cols_buf. */
static int pack(PyObject* seq, Py_ssize_t ncols, const Py_buffer& cb, const Py_buffer& bb) {
    const Py_ssize_t nb = PySequence_Fast_GET_SIZE(seq);
    if (ncols < 0 || cb.len < (Py_ssize_t)(nb * ncols * sizeof(col_rec)) || bb.len < (Py_ssize_t)(nb * sizeof(batch_rec))) {
        PyErr_SetString(PyExc_ValueError, "buffers too small");
        return -1;
    }
    col_rec* C = (col_rec*)cb.buf;
    batch_rec* B = (batch_rec*)bb.buf;
    for (Py_ssize_t b = 0; b < nb; ++b) {
        PyObject* batch = PySequence_Fast_GET_ITEM(seq, b);
        /* RecordBatch keeps its Arrays in _columns (a list, or lazy columns
         * the `columns` property builds) */
        PyObject* cols = PyObject_GetAttr(batch, s__columns);
        if (cols && !PyList_CheckExact(cols)) {
            Py_DECREF(cols);
            cols = PyObject_GetAttr(batch, s_columns);
        }
        if (!cols) return -1;
        PyObject* cseq = PySequence_Fast(cols, "columns must be a sequence");
        Py_DECREF(cols);
        if (!cseq) return -1;
        if (PySequence_Fast_GET_SIZE(cseq) != ncols) {
            Py_DECREF(cseq);
            PyErr_SetString(PyExc_ValueError, "batches do not share a schema");
            return -1;
        }
        col_rec* r = C + b * ncols;
        for (Py_ssize_t i = 0; i < ncols; ++i) {
            PyObject* a = PySequence_Fast_GET_ITEM(cseq, i);
            int64_t t;
            memset(&r[i], 0, sizeof r[i]);
            if (get_i64(a, s_data_type, &t) || get_i64(a, s_length, &r[i].length) ||
                get_i64(a, s_null_count, &r[i].null_count) || get_ptr(a, s_validity, &r[i].validity, s__bo) ||
                get_ptr(a, s_values, &r[i].values, s__vo) || get_ptr(a, s_offsets, &r[i].offsets, s__oo) ||
                get_i64(a, s_offset, &r[i].offset)) {
                Py_DECREF(cseq);
                return -1;
            }
            r[i].type = (int32_t)t;
        }
        Py_DECREF(cseq);
        B[b].num_columns = (int32_t)ncols;
        B[b].reserved = 0;
        B[b].num_rows = ncols ? r[0].length : 0;
        B[b].columns = (uint64_t)(uintptr_t)r;
    }
    return 0;
}

/* pack_host_batches(batches, ncols, cols_buf, batches_buf) -> None
 * cols_buf: writable, >= len(batches) * ncols dfmi_column records;
 * batches_buf: writable, >= len(batches) dfmi_batch records. Each batch's
 * `columns` pointer points into cols_buf. */
static PyObject* pack_host_batches(PyObject* self, PyObject* args) {
    PyObject* batches;
    Py_ssize_t ncols;
    Py_buffer cb, bb;
    if (!PyArg_ParseTuple(args, "Onw*w*", &batches, &ncols, &cb, &bb)) return NULL;
    PyObject* seq = PySequence_Fast(batches, "batches must be a sequence");
    const int rc = seq ? pack(seq, ncols, cb, bb) : -1;
    Py_XDECREF(seq);
    PyBuffer_Release(&cb);
    PyBuffer_Release(&bb);
    if (rc) return NULL;
    Py_RETURN_NONE;
}

static int width_of(int t) {
    switch (t) {
        case 2: case 6: return 1;            /* Int8, UInt8 */
        case 3: case 7: return 2;            /* Int16, UInt16 */
        case 4: case 8: case 10: return 4;   /* Int32, UInt32, Float32 */
        case 5: case 9: case 11: return 8;   /* Int64, UInt64, Float64 */
        default: return 0;
    }
}

static inline int set_ll(PyObject* d, PyObject* k, long long v) {
    PyObject* x = PyLong_FromLongLong(v);
    if (!x) return -1;
    const int rc = PyDict_SetItem(d, k, x);
    Py_DECREF(x);
    return rc;
}

/* A new instance of heap type `cls` with a fresh instance dict (no __init__). */
static PyObject* bare_instance(PyTypeObject* cls, PyObject** dict) {
    PyObject* o = cls->tp_alloc(cls, 0);
    if (!o) return NULL;
    PyObject** dp = _PyObject_GetDictPtr(o);
    if (!dp) {
        Py_DECREF(o);
        PyErr_SetString(PyExc_TypeError, "class without an instance dict");
        return NULL;
    }
    *dp = PyDict_New();
    if (!*dp) {
        Py_DECREF(o);
        return NULL;
    }
    *dict = *dp;
    return o;
}

/* One BlockArray (arrow.py) for an output record: its buffers are byte
 * ranges of `block` (64-byte padded, clamped to the block), each torch view
 * made when first read. */
static PyObject* block_array(PyTypeObject* cls, PyObject* block, uint64_t base, uint64_t size, const out_rec& r,
                             PyObject* dtypes) {
    if (r.type < 0 || r.type >= PyList_GET_SIZE(dtypes)) {
        PyErr_SetString(PyExc_ValueError, "bad output type");
        return NULL;
    }
    PyObject* d;
    PyObject* a = bare_instance(cls, &d);
    if (!a) return NULL;
    const int64_t n = r.length;
    auto range = [&](uint64_t ptr, uint64_t nbytes, PyObject* ko, PyObject* kn) -> int {
        if (ptr < base || ptr > base + size) {
            PyErr_SetString(PyExc_ValueError, "output buffer outside the block");
            return -1;
        }
        const uint64_t o = ptr - base;
        uint64_t len = nbytes < 64 ? 64 : (nbytes + 63) & ~(uint64_t)63;
        if (o + len > size) len = size - o;
        return set_ll(d, ko, (long long)o) || set_ll(d, kn, (long long)len) ? -1 : 0;
    };
    // (`offset` is BlockArray's class attribute 0; a buffer without its range
    // keys -- offsets of a fixed-width array, validity without nulls -- reads
    // as None through its descriptor: fewer dict entries per array)
    int bad = PyDict_SetItem(d, s_data_type, PyList_GET_ITEM(dtypes, r.type)) || set_ll(d, s_length, n) ||
              set_ll(d, s_null_count, r.null_count) || PyDict_SetItem(d, s__blk, block);
    if (!bad) {
        if (r.type == 12) { /* Utf8: offsets + data */
            bad = range(r.offsets, (uint64_t)(n + 1) * 4, s__oo, s__on) ||
                  range(r.data, (uint64_t)r.data_length, s__vo, s__vn);
        } else {
            const uint64_t nb = r.type == 1 ? (uint64_t)(n + 7) / 8 : (uint64_t)n * width_of(r.type);
            bad = range(r.values, nb, s__vo, s__vn);
        }
    }
    if (!bad && r.null_count > 0) bad = range(r.validity, (uint64_t)(n + 7) / 8, s__bo, s__bn);
    if (bad) {
        Py_DECREF(a);
        return NULL;
    }
    return a;
}

/* make_block_batches(batch_cls, array_cls, schema, block, outs, nb, nout, inputs, dtypes) -> list
 * The output RecordBatches of a caller-owned host-batches call
 * (dfmi_filter_project_host_batches_into): `outs` holds nb * nout
 * dfmi_out_column records filled by the library (pointers into `block`, a
 * host uint8 tensor); batch b's column o is a BlockArray over the block, or --
 * passthrough_column >= 0 -- input batch b's own Array (the Arc clone of
 * expression.rs:272-276). One call per group: no per-batch Python. */
static PyObject* make_block_batches(PyObject* self, PyObject* args) {
    PyObject *bcls, *acls, *schema, *block, *inputs, *dtypes;
    Py_buffer ob;
    Py_ssize_t nb, nout;
    if (!PyArg_ParseTuple(args, "O!O!OOy*nnOO!", &PyType_Type, &bcls, &PyType_Type, &acls, &schema, &block, &ob, &nb,
                          &nout, &inputs, &PyList_Type, &dtypes))
        return NULL;
    PyObject* result = NULL;
    PyObject* inseq = NULL;
    do {
        if (!THPVariable_Check(block)) {
            PyErr_SetString(PyExc_TypeError, "block must be a torch.Tensor");
            break;
        }
        const at::Tensor& bt = THPVariable_Unpack(block);
        if (!bt.is_cpu() || !bt.is_contiguous()) {
            PyErr_SetString(PyExc_ValueError, "block must be a contiguous host tensor");
            break;
        }
        const uint64_t base = (uint64_t)(uintptr_t)bt.data_ptr(), size = (uint64_t)bt.nbytes();
        if (nb < 0 || nout < 0 || ob.len < (Py_ssize_t)(nb * nout * sizeof(out_rec))) {
            PyErr_SetString(PyExc_ValueError, "outs too small");
            break;
        }
        inseq = PySequence_Fast(inputs, "inputs must be a sequence");
        if (!inseq) break;
        if (PySequence_Fast_GET_SIZE(inseq) < nb) {
            PyErr_SetString(PyExc_ValueError, "fewer input batches than outputs");
            break;
        }
        const out_rec* R = (const out_rec*)ob.buf;
        result = PyList_New(nb);
        if (!result) break;
        bool fail = false;
        for (Py_ssize_t b = 0; b < nb && !fail; ++b) {
            PyObject* cols = PyList_New(nout);
            if (!cols) {
                fail = true;
                break;
            }
            PyObject* in_cols = NULL;
            for (Py_ssize_t o = 0; o < nout; ++o) {
                const out_rec& r = R[b * nout + o];
                PyObject* a;
                if (r.passthrough_column >= 0) {
                    if (!in_cols) {
                        in_cols = PyObject_GetAttr(PySequence_Fast_GET_ITEM(inseq, b), s_columns);
                        if (!in_cols) {
                            fail = true;
                            break;
                        }
                    }
                    a = PySequence_GetItem(in_cols, r.passthrough_column);
                } else {
                    a = block_array((PyTypeObject*)acls, block, base, size, r, dtypes);
                }
                if (!a) {
                    fail = true;
                    break;
                }
                PyList_SET_ITEM(cols, o, a);
            }
            Py_XDECREF(in_cols);
            PyObject* d;
            PyObject* rb = fail ? NULL : bare_instance((PyTypeObject*)bcls, &d);
            if (!rb || PyDict_SetItem(d, s_schema, schema) || PyDict_SetItem(d, s__columns, cols)) {
                Py_XDECREF(rb);
                Py_DECREF(cols);
                fail = true;
                break;
            }
            Py_DECREF(cols);
            PyList_SET_ITEM(result, b, rb);
        }
        if (fail) Py_CLEAR(result);
    } while (0);
    Py_XDECREF(inseq);
    PyBuffer_Release(&ob);
    return result;
}

static PyMethodDef methods[] = {
    {"make_block_batches", make_block_batches, METH_VARARGS,
     "RecordBatches of BlockArrays over a caller-owned output block (dfmi_filter_project_host_batches_into)."},
    {"pack_host_batches", pack_host_batches, METH_VARARGS,
     "Fill dfmi_column / dfmi_batch records for host batches (include/dfmi.h)."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dfmi_glue", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__dfmi_glue(void) {
#define INTERN(v, s) \
    if (!(v = PyUnicode_InternFromString(s))) return NULL;
    INTERN(s_columns, "columns");
    INTERN(s__columns, "_columns");
    INTERN(s_data_type, "data_type");
    INTERN(s_length, "length");
    INTERN(s_null_count, "null_count");
    INTERN(s_validity, "validity");
    INTERN(s_values, "values");
    INTERN(s_offsets, "offsets");
    INTERN(s_offset, "offset");
    INTERN(s_schema, "schema");
    INTERN(s__blk, "_blk");
    INTERN(s__vo, "_vo");
    INTERN(s__vn, "_vn");
    INTERN(s__bo, "_bo");
    INTERN(s__bn, "_bn");
    INTERN(s__oo, "_oo");
    INTERN(s__on, "_on");
    return PyModule_Create(&module);
}
