/* _resparse: sod_results (include/sod.h) -> Context.results' dict of numpy arrays, in C.
 *
 * The one-image Main.run spends ~20 us of Python after the device finishes turning the staged
 * results into ~22 numpy arrays (_lib._results_from_struct: a ctypes struct read, a copy per
 * memory run and a view per array).  Here each array is allocated and filled by one memcpy
 * straight from the struct's pointers: same dict, same dtypes and shapes, same values (copies,
 * never views of the context's staging buffer).  _lib uses it when it is built and keeps the
 * Python reader otherwise (tests check the two agree).
 *
 *   results(struct_address: int, mask: int) -> dict   (mask: SOD_RES_* bits, as requested)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <string.h>

#include "sod.h"

/* a new array of n rows (w columns when w > 0) filled from src, zeros when src is null */
static PyObject* copy_array(const void* src, int64_t n, int w, int typenum) {
  npy_intp dims[2] = {(npy_intp)(n > 0 ? n : 0), (npy_intp)w};
  PyObject* a = PyArray_SimpleNew(w ? 2 : 1, dims, typenum);
  if (!a) return NULL;
  const size_t bytes = (size_t)PyArray_NBYTES((PyArrayObject*)a);
  if (bytes) {
    if (src)
      memcpy(PyArray_DATA((PyArrayObject*)a), src, bytes);
    else
      memset(PyArray_DATA((PyArrayObject*)a), 0, bytes);
  }
  return a;
}

/* d[key] = copy_array(...), the new reference handed to the dict */
static int put(PyObject* d, const char* key, const void* src, int64_t n, int w, int typenum) {
  PyObject* a = copy_array(src, n, w, typenum);
  if (!a) return -1;
  const int rc = PyDict_SetItemString(d, key, a);
  Py_DECREF(a);
  return rc;
}

static PyObject* results(PyObject* self, PyObject* args) {
  (void)self;
  unsigned long long addr;
  int mask;
  if (!PyArg_ParseTuple(args, "Ki", &addr, &mask)) return NULL;
  if (!addr) {
    PyErr_SetString(PyExc_ValueError, "null sod_results address");
    return NULL;
  }
  const sod_results* r = (const sod_results*)(uintptr_t)addr;
  PyObject* out = PyDict_New();
  PyObject* d = NULL;
  if (!out) return NULL;
  if (mask & SOD_RES_MATCH) {
    PyObject* t = PyTuple_New(4);
    if (!t) goto fail;
    PyObject* m[4] = {copy_array(r->idx1, r->nq, 0, NPY_INT32),
                      copy_array(r->d1, r->nq, 0, NPY_FLOAT32),
                      copy_array(r->d2, r->nq, 0, NPY_FLOAT32),
                      copy_array(r->good, r->nq, 0, NPY_BOOL)};
    for (int i = 0; i < 4; ++i) {
      if (!m[i]) {
        for (int j = 0; j < 4; ++j) Py_XDECREF(m[j]);
        Py_DECREF(t);
        goto fail;
      }
    }
    for (int i = 0; i < 4; ++i) PyTuple_SET_ITEM(t, i, m[i]);   /* (steals) */
    const int rc = PyDict_SetItemString(out, "match", t);
    Py_DECREF(t);
    if (rc) goto fail;
  }
  const int64_t V = r->n_valid, M = r->n_members;
  if (r->selected) {
    if (!(d = PyDict_New())) goto fail;
    if (put(d, "keys", r->keys, V, 4, NPY_INT32) || put(d, "votes", r->votes, V, 0, NPY_INT32) ||
        put(d, "offsets", r->offsets, V + 1, 0, NPY_INT64) ||
        put(d, "members", r->members, M, 0, NPY_INT32) ||
        put(d, "means", r->means, V, 6, NPY_FLOAT64) || PyDict_SetItemString(out, "valid", d))
      goto fail;
    Py_CLEAR(d);
  }
  if (r->affined) {
    if (!(d = PyDict_New())) goto fail;
    if (put(d, "survived", r->survived, V, 0, NPY_BOOL) ||
        put(d, "votes", r->affine_votes, V, 0, NPY_INT32) ||
        put(d, "params", r->params, V, 6, NPY_FLOAT64) ||
        put(d, "alive", r->alive, M, 0, NPY_BOOL) || PyDict_SetItemString(out, "affine", d))
      goto fail;
    Py_CLEAR(d);
  }
  if (r->post) {
    const int64_t nb = r->n_bins, np_ = r->n_pos, no = r->n_ori;
    if (!(d = PyDict_New())) goto fail;
    if (put(d, "bin_index", r->bin_index, nb, 0, NPY_INT32) ||
        put(d, "pos_off", r->pos_off, np_ + 1, 0, NPY_INT32) ||
        put(d, "pos_members", r->pos_members, nb, 0, NPY_INT32) ||
        put(d, "ori_pos_off", r->ori_pos_off, np_ + 1, 0, NPY_INT32) ||
        put(d, "ori_off", r->ori_off, no + 1, 0, NPY_INT32) ||
        put(d, "ori_members", r->ori_members, nb, 0, NPY_INT32) ||
        put(d, "final_orientation", r->final_orientation, np_, 0, NPY_FLOAT64) ||
        put(d, "final_pose", r->final_pose, np_, 6, NPY_FLOAT64) ||
        PyDict_SetItemString(out, "post", d))
      goto fail;
    Py_CLEAR(d);
  }
  return out;
fail:
  Py_XDECREF(d);
  Py_DECREF(out);
  return NULL;
}

static PyMethodDef kMethods[] = {
    {"results", results, METH_VARARGS,
     "results(struct_address, mask) -> dict: sod_results as Context.results' numpy arrays"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_resparse", NULL, -1, kMethods,
                                     NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__resparse(void) {
  import_array();
  return PyModule_Create(&kModule);
}
