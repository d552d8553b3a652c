/* kd_pystr.c — CPython helper for the writer formatting path (host code, no GPU): the per-value
 * str objects of one ASCII output buffer (kd_hex_encode's hex), built straight from the buffer
 * with PyUnicode_New + memcpy — no decode of the whole buffer into one str and no slice object per
 * value.  ascii_slices(buf, lo, hi) -> [buf[lo[i]:hi[i]] as str for every i]; lo / hi are int64
 * buffers of equal length, every range inside buf, every byte < 0x80 (the hex alphabet). */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <string.h>

static PyObject* ascii_slices(PyObject* self, PyObject* args) {
    PyObject *obuf, *olo, *ohi;
    if (!PyArg_ParseTuple(args, "OOO", &obuf, &olo, &ohi)) return NULL;
    Py_buffer b, l, h;
    if (PyObject_GetBuffer(obuf, &b, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if (PyObject_GetBuffer(olo, &l, PyBUF_C_CONTIGUOUS) < 0) { PyBuffer_Release(&b); return NULL; }
    if (PyObject_GetBuffer(ohi, &h, PyBUF_C_CONTIGUOUS) < 0) { PyBuffer_Release(&b); PyBuffer_Release(&l); return NULL; }
    PyObject* out = NULL;
    if (l.len != h.len || l.len % 8) {
        PyErr_SetString(PyExc_ValueError, "ascii_slices: lo and hi must be int64 arrays of one length");
        goto done;
    }
    const Py_ssize_t n = l.len / 8;
    const unsigned char* p = (const unsigned char*)b.buf;
    const long long* lo = (const long long*)l.buf;
    const long long* hi = (const long long*)h.buf;
    out = PyList_New(n);
    if (!out) goto done;
    for (Py_ssize_t i = 0; i < n; i++) {
        const long long a = lo[i], e = hi[i];
        if (a < 0 || e < a || e > (long long)b.len) {
            PyErr_Format(PyExc_ValueError, "ascii_slices: range %zd [%lld, %lld) outside the buffer", i, a, e);
            Py_CLEAR(out);
            goto done;
        }
        PyObject* s = PyUnicode_New((Py_ssize_t)(e - a), 127);
        if (!s) { Py_CLEAR(out); goto done; }
        memcpy(PyUnicode_DATA(s), p + a, (size_t)(e - a));
        PyList_SET_ITEM(out, i, s);
    }
done:
    PyBuffer_Release(&b);
    PyBuffer_Release(&l);
    PyBuffer_Release(&h);
    return out;
}

static PyMethodDef methods[] = {
    {"ascii_slices", ascii_slices, METH_VARARGS, "str per [lo, hi) range of an ASCII buffer"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_kd_pystr", NULL, -1, methods};

PyMODINIT_FUNC PyInit__kd_pystr(void) { return PyModule_Create(&module); }
