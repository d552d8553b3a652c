/* kd_pystr.c — CPython helpers of the drop-in's host side (no GPU):
 *
 * ascii_slices(buf, lo, hi) — the writer formatting path: the per-value str objects of one ASCII
 *   output buffer (kd_hex_encode's hex), built straight from the buffer with PyUnicode_New + memcpy
 *   — no decode of the whole buffer into one str and no slice object per value.  lo / hi are int64
 *   buffers of equal length, every range inside buf, every byte < 0x80 (the hex alphabet).
 *
 * build_deltas(...) — the object side of RichBaseDataset.diff_feature (kart/rich_base_dataset.py:
 *   240-300) for a whole delta list at once: per delta the lazy blob of each present side, the
 *   promise partial(get_feature_from_blob, blob) (kart/base_dataset.py:506-507: no blob is read and
 *   get_feature is not called here), the two KeyValue halves and the Delta
 *   (kart/diff_structs.py:12-40,47-80), built in C with the slots filled directly.
 *
 * attach_fields(...) — the changed_fields of a field diff's updates from kd_fielddiff's mask rows:
 *   one decode per distinct mask, a fresh list per update. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>
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

/* the byte offset of a __slots__ member of a Python class (its member descriptor) */
static Py_ssize_t slot_offset(PyObject* type, const char* name) {
    PyObject* d = PyObject_GetAttrString(type, name);
    if (!d) return -1;
    Py_ssize_t off = -1;
    if (Py_TYPE(d) == &PyMemberDescr_Type) off = ((PyMemberDescrObject*)d)->d_member->offset;
    else PyErr_Format(PyExc_TypeError, "%s is not a __slots__ member", name);
    Py_DECREF(d);
    return off;
}

static inline void set_slot(PyObject* obj, Py_ssize_t off, PyObject* v) {  /* steals v */
    PyObject** p = (PyObject**)((char*)obj + off);
    PyObject* old = *p;
    *p = v;
    Py_XDECREF(old);
}

/* functools.partial(fn, arg) built directly: the partial's func / args / keywords members (their
 * member-descriptor offsets) and its vectorcall entry (the type's tp_vectorcall_offset) filled as
 * partial_new fills them, copied from a template made by the constructor for the same fn. */
typedef struct {
    PyTypeObject* type;
    Py_ssize_t fn, args, kwoff, vc;
    void* vcfunc;
    PyObject* kw;  /* the keywords dict all direct partials of one call share: empty, never written
                    * (Kart reads .keywords of a promise nowhere; partial_call copies it when non-empty) */
    int direct;
} PartialMaker;

static int partial_maker_init(PartialMaker* m, PyObject* pt, PyObject* fn) {
    memset(m, 0, sizeof(*m));
    m->type = (PyTypeObject*)pt;
    if (!fn || fn == Py_None) return 0;
    PyObject* tmpl = PyObject_CallFunctionObjArgs(pt, fn, Py_None, NULL);
    if (!tmpl) return -1;
    m->fn = slot_offset(pt, "func");
    m->args = slot_offset(pt, "args");
    m->kwoff = slot_offset(pt, "keywords");
    if (m->fn < 0 || m->args < 0 || m->kwoff < 0) {
        PyErr_Clear();  /* not CPython's partial layout: go through the constructor */
        Py_DECREF(tmpl);
        return 0;
    }
    m->vc = m->type->tp_vectorcall_offset;
    PyObject** f = (PyObject**)((char*)tmpl + m->fn);
    PyObject** a = (PyObject**)((char*)tmpl + m->args);
    PyObject** k = (PyObject**)((char*)tmpl + m->kwoff);
    m->direct = Py_TYPE(tmpl) == m->type && *f == fn && PyTuple_CheckExact(*a) && PyTuple_GET_SIZE(*a) == 1 &&
                PyTuple_GET_ITEM(*a, 0) == Py_None && PyDict_CheckExact(*k) && PyDict_GET_SIZE(*k) == 0 &&
                m->type->tp_dictoffset >= 0;
    if (m->vc > 0) m->vcfunc = *(void**)((char*)tmpl + m->vc);
    Py_DECREF(tmpl);
    if (m->direct && !(m->kw = PyDict_New())) return -1;
    return 0;
}

static PyObject* partial_make(const PartialMaker* m, PyObject* fn, PyObject* arg) {
    if (!m->direct) return PyObject_CallFunctionObjArgs((PyObject*)m->type, fn, arg, NULL);
    PyObject* args = PyTuple_Pack(1, arg);
    PyObject* p = m->type->tp_alloc(m->type, 0);
    if (!args || !p) {
        Py_XDECREF(args); Py_XDECREF(p);
        return NULL;
    }
    PyObject* kw = m->kw;
    Py_INCREF(kw);
    Py_INCREF(fn);
    set_slot(p, m->fn, fn);
    set_slot(p, m->args, args);
    set_slot(p, m->kwoff, kw);
    if (m->vc > 0) *(void**)((char*)p + m->vc) = m->vcfunc;
    return p;
}

/* pk i of an int64 buffer or a list */
static PyObject* pk_at(PyObject* list, const long long* arr, Py_ssize_t i) {
    if (list) {
        PyObject* x = PyList_GET_ITEM(list, i);
        Py_INCREF(x);
        return x;
    }
    return PyLong_FromLongLong(arr[i]);
}

/* ---- Promise: partial(get_feature_from_blob, blob) with the blob made on first use ----
 * What a delta half's value is (kart/base_dataset.py:506-507 promise, base_diff_writer.py:506 reads
 * `value.args[0]`): calling it returns func(blob); .args = (blob,), .func, .keywords as a partial
 * has.  The LazyBlob (blob_type(src, i)) is created the first time the value or .args is used, so a
 * diff builds one object per delta half here instead of three (blob, partial, args tuple) plus the
 * leaf-index int. */
typedef struct {
    PyObject_HEAD
    PyObject* func;
    PyObject* src;
    PyObject* blob_type;
    PyObject* blob;
    long long i;
} Promise;

static PyTypeObject PromiseType;

static PyObject* promise_blob(Promise* p) {
    if (!p->blob) p->blob = PyObject_CallFunction(p->blob_type, "OL", p->src, p->i);
    return p->blob;  /* borrowed; NULL on error */
}

static PyObject* promise_call(PyObject* self, PyObject* args, PyObject* kw) {
    Promise* p = (Promise*)self;
    PyObject* blob = promise_blob(p);
    if (!blob) return NULL;
    const Py_ssize_t na = PyTuple_GET_SIZE(args);
    if (na == 0 && (!kw || PyDict_GET_SIZE(kw) == 0)) return PyObject_CallOneArg(p->func, blob);
    PyObject* all = PyTuple_New(na + 1);
    if (!all) return NULL;
    Py_INCREF(blob);
    PyTuple_SET_ITEM(all, 0, blob);
    for (Py_ssize_t k = 0; k < na; k++) {
        PyObject* x = PyTuple_GET_ITEM(args, k);
        Py_INCREF(x);
        PyTuple_SET_ITEM(all, k + 1, x);
    }
    PyObject* r = PyObject_Call(p->func, all, kw);
    Py_DECREF(all);
    return r;
}

static PyObject* promise_get_args(PyObject* self, void* c) {
    PyObject* blob = promise_blob((Promise*)self);
    return blob ? PyTuple_Pack(1, blob) : NULL;
}

static PyObject* promise_get_func(PyObject* self, void* c) {
    Py_INCREF(((Promise*)self)->func);
    return ((Promise*)self)->func;
}

static PyObject* promise_get_keywords(PyObject* self, void* c) { return PyDict_New(); }

static PyObject* promise_repr(PyObject* self) {
    PyObject* blob = promise_blob((Promise*)self);
    if (!blob) return NULL;
    return PyUnicode_FromFormat("functools.partial(%R, %R)", ((Promise*)self)->func, blob);
}

static int promise_traverse(PyObject* self, visitproc visit, void* arg) {
    Promise* p = (Promise*)self;
    Py_VISIT(p->func);
    Py_VISIT(p->src);
    Py_VISIT(p->blob_type);
    Py_VISIT(p->blob);
    return 0;
}

static int promise_clear(PyObject* self) {
    Promise* p = (Promise*)self;
    Py_CLEAR(p->func);
    Py_CLEAR(p->src);
    Py_CLEAR(p->blob_type);
    Py_CLEAR(p->blob);
    return 0;
}

static void promise_dealloc(PyObject* self) {
    PyObject_GC_UnTrack(self);
    promise_clear(self);
    Py_TYPE(self)->tp_free(self);
}

static PyGetSetDef promise_getset[] = {
    {"args", promise_get_args, NULL, "(blob,): the promise's one argument", NULL},
    {"func", promise_get_func, NULL, "the getter the blob is passed to", NULL},
    {"keywords", promise_get_keywords, NULL, "always empty", NULL},
    {NULL, NULL, NULL, NULL, NULL},
};

static PyTypeObject PromiseType = {
    PyVarObject_HEAD_INIT(NULL, 0)
    .tp_name = "kart_amd._kd_pystr.Promise",
    .tp_basicsize = sizeof(Promise),
    .tp_dealloc = promise_dealloc,
    .tp_repr = promise_repr,
    .tp_call = promise_call,
    .tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC,
    .tp_doc = "partial(get_feature_from_blob, blob) whose blob is made on first use",
    .tp_traverse = promise_traverse,
    .tp_clear = promise_clear,
    .tp_getset = promise_getset,
};

/* build_deltas(delta_type, kv_type, blob_type, partial_type, old_get, new_get, old_src, new_src,
 *              old_leaf, new_leaf, old_pk, new_pk, own)
 * old_leaf / new_leaf: int64 buffers of n leaf indices (-1: the side is absent); old_pk / new_pk: int64
 * buffers or lists of n pks (entries of absent sides unused).  own: delta_type / kv_type are
 * kart_amd.deltas' own classes (Delta filled field by field, KeyValue's slots directly), else the
 * halves are (pk, promise) tuples passed to delta_type(old, new).  blob_type is kart_amd.dataset's
 * LazyBlob (slots _src, _i, _data).
 * Returns (keys, deltas, upd_rows, upd_deltas, upd_keys): the key of each delta (old pk, else new pk)
 * and the delta, and the updates' row numbers (bytes: native int64, no int object per row), deltas
 * and keys.  out (optional dict): each delta is
 * also stored there at its key (a DeltaDiff's dict filled in place). */
static PyObject* build_deltas(PyObject* self, PyObject* args) {
    PyObject *dt, *kvt, *bt, *pt, *og, *ng, *os_, *ns, *ol_o, *nl_o, *op_o, *np_o, *out = Py_None;
    int own;
    if (!PyArg_ParseTuple(args, "OOOOOOOOOOOOp|O", &dt, &kvt, &bt, &pt, &og, &ng, &os_, &ns, &ol_o, &nl_o, &op_o, &np_o, &own,
                          &out))
        return NULL;
    if (out != Py_None && !PyDict_Check(out)) {
        PyErr_SetString(PyExc_TypeError, "build_deltas: out must be a dict");
        return NULL;
    }
    PyObject* const out_dict = out != Py_None ? out : NULL;
    Py_buffer ol = {0}, nl = {0}, opb = {0}, npb = {0};
    PyObject *keys = NULL, *dl = NULL, *urows = NULL, *udl = NULL, *ukeys = NULL, *ret = NULL;
    long long* ur = NULL;  /* the updates' rows */
    Py_ssize_t nur = 0;
    PyObject *t_ins = NULL, *t_upd = NULL, *t_del = NULL;
    PartialMaker pm[2];
    memset(pm, 0, sizeof(pm));
    PyObject *zero = NULL;
    if (PyObject_GetBuffer(ol_o, &ol, PyBUF_C_CONTIGUOUS) < 0) goto fail;
    if (PyObject_GetBuffer(nl_o, &nl, PyBUF_C_CONTIGUOUS) < 0) goto fail;
    const Py_ssize_t n = ol.len / 8;
    if (ol.len != nl.len || ol.len % 8) { PyErr_SetString(PyExc_ValueError, "build_deltas: leaf arrays"); goto fail; }
    PyObject* op_list = PyList_Check(op_o) ? op_o : NULL;
    PyObject* np_list = PyList_Check(np_o) ? np_o : NULL;
    if (!op_list && PyObject_GetBuffer(op_o, &opb, PyBUF_C_CONTIGUOUS) < 0) goto fail;
    if (!np_list && PyObject_GetBuffer(np_o, &npb, PyBUF_C_CONTIGUOUS) < 0) goto fail;
    if ((op_list ? PyList_GET_SIZE(op_list) : opb.len / 8) != n || (np_list ? PyList_GET_SIZE(np_list) : npb.len / 8) != n) {
        PyErr_SetString(PyExc_ValueError, "build_deltas: pk arrays");
        goto fail;
    }
    const long long* olp = (const long long*)ol.buf;
    const long long* nlp = (const long long*)nl.buf;
    const long long* opp = (const long long*)opb.buf;
    const long long* npp = (const long long*)npb.buf;
    const Py_ssize_t b_src = slot_offset(bt, "_src"), b_i = slot_offset(bt, "_i"), b_data = slot_offset(bt, "_data");
    if (b_src < 0 || b_i < 0 || b_data < 0) goto fail;
    Py_ssize_t kv_key = -1, kv_val = -1, d_old = -1, d_new = -1, d_type = -1, d_flags = -1;
    if (own) {
        kv_key = slot_offset(kvt, "key");
        kv_val = slot_offset(kvt, "value");
        d_old = slot_offset(dt, "old");
        d_new = slot_offset(dt, "new");
        d_type = slot_offset(dt, "type");
        d_flags = slot_offset(dt, "flags");
        if (kv_key < 0 || kv_val < 0 || d_old < 0 || d_new < 0 || d_type < 0 || d_flags < 0) goto fail;
    }
    const int promise_mode = pt == (PyObject*)&PromiseType;  /* lazy-blob promises, else functools.partial */
    if (!promise_mode && (partial_maker_init(&pm[0], pt, og) < 0 || partial_maker_init(&pm[1], pt, ng) < 0)) goto fail;
    t_ins = PyUnicode_InternFromString("insert"); t_upd = PyUnicode_InternFromString("update");
    t_del = PyUnicode_InternFromString("delete");
    zero = PyLong_FromLong(0);
    if (!t_ins || !t_upd || !t_del || !zero) goto fail;
    keys = PyList_New(n); dl = PyList_New(n);
    udl = PyList_New(0); ukeys = PyList_New(0);
    ur = (long long*)PyMem_Malloc(sizeof(long long) * (size_t)(n ? n : 1));
    if (!keys || !dl || !udl || !ukeys || !ur) { if (!PyErr_Occurred()) PyErr_NoMemory(); goto fail; }
    PyTypeObject* BT = (PyTypeObject*)bt;
    PyTypeObject* KT = (PyTypeObject*)kvt;
    PyTypeObject* DT = (PyTypeObject*)dt;
    for (Py_ssize_t i = 0; i < n; i++) {
        PyObject* half[2] = {NULL, NULL};
        PyObject* pkv[2] = {NULL, NULL};
        const long long leaf[2] = {olp[i], nlp[i]};
        if (leaf[0] < 0 && leaf[1] < 0) {
            PyErr_Format(PyExc_ValueError, "build_deltas: row %zd has neither side (Empty Delta)", i);
            goto fail;
        }
        for (int s = 0; s < 2; s++) {
            if (leaf[s] < 0) continue;
            PyObject* pk;
            if (s && pkv[0] && !np_list && !op_list && npp[i] == opp[i]) {  /* an update: one int for both keys */
                pk = pkv[0];
                Py_INCREF(pk);
            } else {
                pk = pk_at(s ? np_list : op_list, s ? npp : opp, i);
            }
            PyObject* src = s ? ns : os_;
            PyObject* promise;
            if (promise_mode) {
                Promise* pr = pk ? (Promise*)PromiseType.tp_alloc(&PromiseType, 0) : NULL;
                if (!pr) { Py_XDECREF(pk); goto item_fail; }
                PyObject* fn = s ? ng : og;
                Py_INCREF(fn); pr->func = fn;
                Py_INCREF(src); pr->src = src;
                Py_INCREF(bt); pr->blob_type = bt;
                pr->i = leaf[s];
                promise = (PyObject*)pr;
            } else {
                PyObject* blob = BT->tp_alloc(BT, 0);
                PyObject* li = PyLong_FromLongLong(leaf[s]);
                if (!pk || !blob || !li) { Py_XDECREF(pk); Py_XDECREF(blob); Py_XDECREF(li); goto item_fail; }
                Py_INCREF(src);
                set_slot(blob, b_src, src);
                set_slot(blob, b_i, li);
                Py_INCREF(Py_None);
                set_slot(blob, b_data, Py_None);
                promise = partial_make(&pm[s], s ? ng : og, blob);
                Py_DECREF(blob);
                if (!promise) { Py_DECREF(pk); goto item_fail; }
            }
            pkv[s] = pk;
            if (own) {
                PyObject* kv = KT->tp_alloc(KT, 0);
                if (!kv) { Py_DECREF(promise); goto item_fail; }
                Py_INCREF(pk);
                set_slot(kv, kv_key, pk);
                set_slot(kv, kv_val, promise);
                half[s] = kv;
            } else {
                half[s] = PyTuple_Pack(2, pk, promise);
                Py_DECREF(promise);
                if (!half[s]) goto item_fail;
            }
            continue;
        item_fail:
            Py_XDECREF(half[0]); Py_XDECREF(half[1]); Py_XDECREF(pkv[0]); Py_XDECREF(pkv[1]);
            goto fail;
        }
        PyObject* d;
        if (own) {
            d = DT->tp_alloc(DT, 0);
            if (!d) { Py_XDECREF(half[0]); Py_XDECREF(half[1]); Py_XDECREF(pkv[0]); Py_XDECREF(pkv[1]); goto fail; }
            PyObject* ty = !half[0] ? t_ins : !half[1] ? t_del : t_upd;
            Py_INCREF(ty);
            set_slot(d, d_type, ty);
            Py_INCREF(zero);
            set_slot(d, d_flags, zero);
            set_slot(d, d_old, half[0] ? half[0] : (Py_INCREF(Py_None), Py_None));
            set_slot(d, d_new, half[1] ? half[1] : (Py_INCREF(Py_None), Py_None));
            half[0] = half[1] = NULL;  /* owned by the delta now */
        } else {
            d = PyObject_CallFunctionObjArgs(dt, half[0] ? half[0] : Py_None, half[1] ? half[1] : Py_None, NULL);
            if (!d) { Py_XDECREF(half[0]); Py_XDECREF(half[1]); Py_XDECREF(pkv[0]); Py_XDECREF(pkv[1]); goto fail; }
        }
        Py_XDECREF(half[0]);
        Py_XDECREF(half[1]);
        PyObject* key = pkv[0] ? pkv[0] : pkv[1];
        if (out_dict && PyDict_SetItem(out_dict, key, d) < 0) {
            Py_DECREF(d); Py_XDECREF(pkv[0]); Py_XDECREF(pkv[1]);
            goto fail;
        }
        Py_INCREF(key);
        PyList_SET_ITEM(keys, i, key);
        Py_INCREF(d);
        PyList_SET_ITEM(dl, i, d);
        if (pkv[0] && pkv[1]) {
            ur[nur++] = i;
            if (PyList_Append(udl, d) < 0 || PyList_Append(ukeys, pkv[0]) < 0) {
                Py_DECREF(d); Py_XDECREF(pkv[0]); Py_XDECREF(pkv[1]);
                goto fail;
            }
        }
        Py_DECREF(d);
        Py_XDECREF(pkv[0]);
        Py_XDECREF(pkv[1]);
    }
    urows = PyBytes_FromStringAndSize((const char*)ur, (Py_ssize_t)(sizeof(long long) * (size_t)nur));
    if (urows) ret = PyTuple_Pack(5, keys, dl, urows, udl, ukeys);
fail:
    PyMem_Free(ur);
    Py_XDECREF(keys); Py_XDECREF(dl); Py_XDECREF(urows); Py_XDECREF(udl); Py_XDECREF(ukeys);
    Py_XDECREF(t_ins); Py_XDECREF(t_upd); Py_XDECREF(t_del); Py_XDECREF(zero);
    Py_XDECREF(pm[0].kw); Py_XDECREF(pm[1].kw);
    if (ol.obj) PyBuffer_Release(&ol);
    if (nl.obj) PyBuffer_Release(&nl);
    if (opb.obj) PyBuffer_Release(&opb);
    if (npb.obj) PyBuffer_Release(&npb);
    return ret;
}

/* attach_fields(deltas, masks, status, words, names_of, delta_type) — the changed_fields of every
 * update of a field diff (kart_amd/dataset.py field_diff): delta i gets a fresh list of the names
 * mask row i (words uint64 per row) stands for, or None where status[i] (uint8) is not 0.  The rows'
 * distinct masks (a layer's updates share a handful) are found with an open-addressing table over
 * the mask words and decoded once each by names_of(i) -> list (i: the first row holding that mask).
 * Deltas of exactly delta_type get the changed_fields slot written directly; any other object goes
 * through setattr.  Returns the number of distinct masks. */
typedef struct {
    Py_ssize_t row;  /* first row of this mask; -1: empty */
    PyObject* names;
} MaskEntry;

static unsigned long long mask_hash(const unsigned long long* w, Py_ssize_t words) {
    unsigned long long h = 0x9E3779B97F4A7C15ull;
    for (Py_ssize_t k = 0; k < words; k++) {
        h ^= w[k];
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    return h;
}

static PyObject* attach_fields(PyObject* self, PyObject* args) {
    PyObject *dl, *om, *os_, *names_of, *dt;
    Py_ssize_t words;
    if (!PyArg_ParseTuple(args, "OOOnOO", &dl, &om, &os_, &words, &names_of, &dt)) return NULL;
    if (!PyList_Check(dl) || words < 1) {
        PyErr_SetString(PyExc_TypeError, "attach_fields: deltas must be a list and words >= 1");
        return NULL;
    }
    Py_buffer mb = {0}, sb = {0};
    MaskEntry* tab = NULL;
    size_t cap = 0, used = 0;
    PyObject *attr = NULL, *ret = NULL;
    if (PyObject_GetBuffer(om, &mb, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if (PyObject_GetBuffer(os_, &sb, PyBUF_C_CONTIGUOUS) < 0) goto done;
    const Py_ssize_t n = PyList_GET_SIZE(dl);
    if (mb.itemsize != 8 || sb.itemsize != 1 || mb.len < (Py_ssize_t)(8 * words) * n || sb.len < n) {
        PyErr_SetString(PyExc_ValueError, "attach_fields: masks must be uint64 and status uint8, one row per delta");
        goto done;
    }
    const unsigned long long* m = (const unsigned long long*)mb.buf;
    const unsigned char* st = (const unsigned char*)sb.buf;
    Py_ssize_t d_cf = -1;
    if (PyType_Check(dt)) {
        d_cf = slot_offset(dt, "changed_fields");
        if (d_cf < 0) PyErr_Clear();  /* no such slot: setattr for every delta */
    }
    attr = PyUnicode_InternFromString("changed_fields");
    cap = 64;
    tab = (MaskEntry*)PyMem_Malloc(cap * sizeof(MaskEntry));
    if (!attr || !tab) { if (!PyErr_Occurred()) PyErr_NoMemory(); goto done; }
    for (size_t k = 0; k < cap; k++) tab[k].row = -1, tab[k].names = NULL;
    for (Py_ssize_t i = 0; i < n; i++) {
        PyObject* v;
        if (st[i]) {
            v = Py_None;
            Py_INCREF(v);
        } else {
            const unsigned long long* w = m + i * words;
            size_t h = (size_t)mask_hash(w, words) & (cap - 1);
            while (tab[h].row >= 0 && memcmp(m + tab[h].row * words, w, 8 * (size_t)words)) h = (h + 1) & (cap - 1);
            if (tab[h].row < 0) {
                PyObject* nm = PyObject_CallFunction(names_of, "n", i);
                if (!nm) goto done;
                if (!PyList_Check(nm)) {
                    Py_DECREF(nm);
                    PyErr_SetString(PyExc_TypeError, "attach_fields: names_of must return a list");
                    goto done;
                }
                tab[h].row = i;
                tab[h].names = nm;
                if (2 * ++used > cap) {  /* grow: rehash every entry into twice the table */
                    const size_t nc = 2 * cap;
                    MaskEntry* nt = (MaskEntry*)PyMem_Malloc(nc * sizeof(MaskEntry));
                    if (!nt) { PyErr_NoMemory(); goto done; }
                    for (size_t k = 0; k < nc; k++) nt[k].row = -1, nt[k].names = NULL;
                    for (size_t k = 0; k < cap; k++) {
                        if (tab[k].row < 0) continue;
                        size_t g = (size_t)mask_hash(m + tab[k].row * words, words) & (nc - 1);
                        while (nt[g].row >= 0) g = (g + 1) & (nc - 1);
                        nt[g] = tab[k];
                    }
                    PyMem_Free(tab);
                    tab = nt;
                    cap = nc;
                    h = (size_t)mask_hash(w, words) & (cap - 1);
                    while (tab[h].row != i) h = (h + 1) & (cap - 1);
                }
            }
            PyObject* src = tab[h].names;
            v = PyList_GetSlice(src, 0, PyList_GET_SIZE(src));
            if (!v) goto done;
        }
        PyObject* d = PyList_GET_ITEM(dl, i);
        if (d_cf >= 0 && Py_TYPE(d) == (PyTypeObject*)dt) {
            set_slot(d, d_cf, v);
        } else {
            const int e = PyObject_SetAttr(d, attr, v);
            Py_DECREF(v);
            if (e < 0) goto done;
        }
    }
    ret = PyLong_FromSize_t(used);
done:
    if (tab)
        for (size_t k = 0; k < cap; k++) Py_XDECREF(tab[k].names);
    PyMem_Free(tab);
    Py_XDECREF(attr);
    if (mb.obj) PyBuffer_Release(&mb);
    if (sb.obj) PyBuffer_Release(&sb);
    return ret;
}

static PyMethodDef methods[] = {
    {"ascii_slices", ascii_slices, METH_VARARGS, "str per [lo, hi) range of an ASCII buffer"},
    {"build_deltas", build_deltas, METH_VARARGS, "Delta objects with lazy promises for a whole delta list"},
    {"attach_fields", attach_fields, METH_VARARGS, "changed_fields of every update from its mask row"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_kd_pystr", NULL, -1, methods};

PyMODINIT_FUNC PyInit__kd_pystr(void) {
    if (PyType_Ready(&PromiseType) < 0) return NULL;
    PyObject* m = PyModule_Create(&module);
    if (!m) return NULL;
    Py_INCREF(&PromiseType);
    if (PyModule_AddObject(m, "Promise", (PyObject*)&PromiseType) < 0) {
        Py_DECREF(&PromiseType);
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
