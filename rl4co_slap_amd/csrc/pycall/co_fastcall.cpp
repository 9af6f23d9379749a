// Fast Python -> C-ABI call path for the env loop (replaces ctypes' per-call argument
// marshalling, ~4 us per 16-argument call, with a METH_FASTCALL conversion, ~0.3 us).
//
// invoke(fn_address, kinds, *args) calls `int fn(...)` where kinds[i] classifies argument
// i: 'i' integer class (int32/int64/uint64/pointer: a Python int, bool or None -> 0),
// 'f' float, 'd' double.  On x86-64 System V, integer-class arguments take the general
// registers and then the stack in their own order and float-class arguments the SSE
// registers in theirs, independently of how the two classes interleave; so one
// trampoline typed (24 x int64, 8 x double) reaches every entry point of include/co_env.h:
// surplus integer slots and registers are ignored by the callee, a `float` parameter reads
// the low 32 bits of its SSE register (the float's bits are placed there), an int32 one the
// low 32 bits of its register / stack slot.  No torch types, no Python objects cross.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>

#if !defined(__x86_64__) || defined(_WIN32)
#error "co_fastcall relies on the x86-64 System V calling convention"
#endif

namespace {

constexpr int kMaxInt = 24, kMaxFp = 8;
typedef int (*Tramp)(int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                     int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                     int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                     double, double, double, double, double, double, double, double);

PyObject* invoke(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs < 2) {
    PyErr_SetString(PyExc_TypeError, "invoke(fn_address, kinds, *args)");
    return nullptr;
  }
  const uint64_t addr = PyLong_AsUnsignedLongLongMask(args[0]);
  if (PyErr_Occurred()) return nullptr;
  Py_ssize_t nk = 0;
  const char* kinds = PyBytes_Check(args[1]) ? PyBytes_AS_STRING(args[1]) : nullptr;
  if (!kinds) {
    PyErr_SetString(PyExc_TypeError, "kinds must be bytes");
    return nullptr;
  }
  nk = PyBytes_GET_SIZE(args[1]);
  if (nk != nargs - 2) {
    PyErr_Format(PyExc_TypeError, "expected %zd arguments, got %zd", nk, nargs - 2);
    return nullptr;
  }
  int64_t iv[kMaxInt] = {0};
  double fv[kMaxFp] = {0.0};
  int ni = 0, nf = 0;
  for (Py_ssize_t k = 0; k < nk; ++k) {
    PyObject* o = args[2 + k];
    const char c = kinds[k];
    if (c == 'i') {
      if (ni == kMaxInt) goto too_many;
      iv[ni++] = o == Py_None ? 0 : (int64_t)PyLong_AsUnsignedLongLongMask(o);
    } else if (c == 'f' || c == 'd') {
      if (nf == kMaxFp) goto too_many;
      const double d = PyFloat_AsDouble(o);
      if (c == 'd') {
        fv[nf++] = d;
      } else {  // the float's bits in the low half of the SSE register
        const float f = (float)d;
        uint64_t u = 0;
        std::memcpy(&u, &f, 4);
        double x;
        std::memcpy(&x, &u, 8);
        fv[nf++] = x;
      }
    } else {
      PyErr_Format(PyExc_ValueError, "bad kind '%c'", c);
      return nullptr;
    }
    if (PyErr_Occurred()) return nullptr;
  }
  {
    const Tramp fn = reinterpret_cast<Tramp>(static_cast<uintptr_t>(addr));
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(iv[0], iv[1], iv[2], iv[3], iv[4], iv[5], iv[6], iv[7], iv[8], iv[9], iv[10], iv[11],
            iv[12], iv[13], iv[14], iv[15], iv[16], iv[17], iv[18], iv[19], iv[20], iv[21],
            iv[22], iv[23], fv[0], fv[1], fv[2], fv[3], fv[4], fv[5], fv[6], fv[7]);
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
  }
too_many:
  PyErr_SetString(PyExc_TypeError, "too many arguments of one class");
  return nullptr;
}

PyMethodDef methods[] = {
    {"invoke", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(invoke)),
     METH_FASTCALL, "invoke(fn_address, kinds, *args) -> int status"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_co_fastcall",
                      "x86-64 SysV fast call path for the co_env C ABI", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__co_fastcall(void) { return PyModule_Create(&module); }
