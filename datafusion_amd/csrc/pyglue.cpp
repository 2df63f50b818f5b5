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

static PyObject *s_columns, *s__columns, *s_data_type, *s_length, *s_null_count, *s_validity, *s_values,
    *s_offsets, *s_offset;

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
 * unless the tensor is in host memory. */
static int get_ptr(PyObject* a, PyObject* name, uint64_t* out) {
    PyObject** dp = _PyObject_GetDictPtr(a);
    PyObject* t = dp && *dp ? PyDict_GetItemWithError(*dp, name) : NULL;
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
                get_i64(a, s_null_count, &r[i].null_count) || get_ptr(a, s_validity, &r[i].validity) ||
                get_ptr(a, s_values, &r[i].values) || get_ptr(a, s_offsets, &r[i].offsets) ||
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

static PyMethodDef methods[] = {
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
    return PyModule_Create(&module);
}
