// Host glue of the drop-in decode loop's per-step calls: one
// METH_FASTCALL entry per fused step that checks the operands, allocates the step's fresh
// output tensors on torch's caching allocator, queues the C-ABI launch on the device's
// current stream and hands the outputs back -- what envs/tsp.py:decode_and_step does in
// Python around co_tsp_decode_step, without ~10 Python-level tensor allocations and
// attribute reads per step.  The C ABI (include/co_env.h) stays the boundary: the entry
// point is called through the address _native resolved from libco_env.so, so this module
// links no kernel code and no library symbols of its own.
//
// Returns None whenever the fast path does not apply (the Python path then runs as before,
// with the same checks and errors), so it never changes behaviour, only host time.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>

#include "co_env.h"

namespace {

using TspDecodeStep = decltype(&co_tsp_decode_step);
using DecodeStep = decltype(&co_decode_step);
using CvrpStep = decltype(&co_cvrp_step);

inline bool is_tensor(PyObject* o) { return o != Py_None && THPVariable_Check(o); }

template <class F>
F fn_at(PyObject* o) {
  return reinterpret_cast<F>(static_cast<uintptr_t>(PyLong_AsUnsignedLongLongMask(o)));
}

// t is on dev, of dtype dt, contiguous, with numel elements (numel < 0: any)
inline bool fits(const at::Tensor& t, const c10::Device& dev, at::ScalarType dt,
                 int64_t numel = -1) {
  return t.device() == dev && t.scalar_type() == dt && t.is_contiguous() &&
         (numel < 0 || t.numel() == numel);
}

inline void* current_stream(const c10::Device& dev) {
  return c10::hip::getCurrentHIPStream(dev.index()).stream();
}

PyObject* wrap_all(std::initializer_list<at::Tensor*> ts) {
  PyObject* out = PyTuple_New((Py_ssize_t)ts.size());
  if (!out) return nullptr;
  Py_ssize_t k = 0;
  for (at::Tensor* t : ts) {
    PyObject* o = t->defined() ? THPVariable_Wrap(std::move(*t)) : (Py_INCREF(Py_None), Py_None);
    if (!o) {
      Py_DECREF(out);
      return nullptr;
    }
    PyTuple_SET_ITEM(out, k++, o);
  }
  return out;
}

// the step's outputs: one storage, carved into the tensors (each a fresh, contiguous,
// non-overlapping region, 256-byte aligned as the caching allocator's blocks are, so the
// kernels' vector paths apply -- as separate allocations would be, at one allocator call)
constexpr int64_t kAlign = 256;
struct Carve {
  at::Tensor chunk;
  int64_t off = 0;
  at::Tensor take(at::IntArrayRef sizes, at::ScalarType dt) {
    const int64_t es = (int64_t)c10::elementSize(dt);
    off = (off + kAlign - 1) & ~(kAlign - 1);
    int64_t n = 1;
    for (auto s : sizes) n *= s;
    auto t = at::empty({0}, chunk.options().dtype(dt));
    t.set_(chunk.storage(), off / es, sizes);
    off += n * es;
    return t;
  }
};

int64_t carve_bytes(std::initializer_list<int64_t> parts) {
  int64_t s = 0;
  for (auto p : parts) s = ((s + kAlign - 1) & ~(kAlign - 1)) + p;
  return s;
}

// tsp_decode_step(fn, logits, mask, i, first_in, action_in, status, clip, temp, mode,
//                 seed, offset, take) -> (act, logp, mask_out, i_out, first_out, done,
//                 reward) | None
// fn: address of co_tsp_decode_step; first_in / action_in: tensor or None.
PyObject* tsp_decode_step(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 13) {
    PyErr_SetString(PyExc_TypeError, "tsp_decode_step: 13 arguments");
    return nullptr;
  }
  if (!is_tensor(a[1]) || !is_tensor(a[2]) || !is_tensor(a[3]) || !is_tensor(a[6]))
    Py_RETURN_NONE;
  const auto fn = fn_at<TspDecodeStep>(a[0]);
  const at::Tensor& logits = THPVariable_Unpack(a[1]);
  const at::Tensor& mask = THPVariable_Unpack(a[2]);
  const at::Tensor& i = THPVariable_Unpack(a[3]);
  const at::Tensor& status = THPVariable_Unpack(a[6]);
  const bool has_first = is_tensor(a[4]), has_ain = is_tensor(a[5]);
  const double clip = PyFloat_AsDouble(a[7]), temp = PyFloat_AsDouble(a[8]);
  const long mode = PyLong_AsLong(a[9]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[10]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[11]);
  const long take = PyLong_AsLong(a[12]);
  if (PyErr_Occurred()) return nullptr;
  // the conditions envs/tsp.py:decode_and_step checks before its launch
  const c10::Device dev = mask.device();
  if (!dev.is_cuda() || logits.device() != dev || i.device() != dev || status.device() != dev ||
      logits.scalar_type() != at::kFloat || logits.dim() != 2 || logits.stride(1) != 1 ||
      mask.dim() != 2 || mask.scalar_type() != at::kBool || !mask.is_contiguous() ||
      i.scalar_type() != at::kLong || !i.is_contiguous() || status.scalar_type() != at::kInt)
    Py_RETURN_NONE;
  const int64_t b = mask.size(0), nl = mask.size(1);
  if (logits.size(0) != b || logits.size(1) != nl || nl > 2048 || i.numel() != b)
    Py_RETURN_NONE;
  const at::Tensor* first = nullptr;
  if (has_first && !take) {
    first = &THPVariable_Unpack(a[4]);
    if (first->device() != dev || first->scalar_type() != at::kLong || !first->is_contiguous() ||
        first->numel() != b)
      Py_RETURN_NONE;
  } else if (!take) {
    Py_RETURN_NONE;
  }
  const at::Tensor* ain = nullptr;
  if (has_ain) {
    ain = &THPVariable_Unpack(a[5]);
    if (ain->device() != dev || ain->scalar_type() != at::kLong || !ain->is_contiguous() ||
        ain->numel() != b)
      Py_RETURN_NONE;
  }
  try {
    // the decoding strategy keeps every step's action and log-probability, the env only
    // the latest state: two chunks, so a kept action does not pin a stale mask
    Carve k, c;
    k.chunk = at::empty({carve_bytes({8 * b, 4 * b})}, mask.options().dtype(at::kByte));
    c.chunk = at::empty({carve_bytes({b * nl, 8 * b, 8 * b, b, b})},
                        mask.options().dtype(at::kByte));
    at::Tensor act = k.take({b}, at::kLong), logp = k.take({b}, at::kFloat);
    at::Tensor mask_out = c.take({b, nl}, at::kBool), i_out = c.take(i.sizes(), at::kLong);
    at::Tensor first_out = c.take({b}, at::kLong), done = c.take({b}, at::kBool);
    at::Tensor reward = c.take({b}, at::kBool);
    void* stream = current_stream(dev);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, nl, logits.const_data_ptr<float>(), logits.stride(0),
            static_cast<const uint8_t*>(mask.const_data_ptr()), (float)clip, (float)temp,
            (int)mode, ain ? ain->const_data_ptr<int64_t>() : nullptr,
            act.mutable_data_ptr<int64_t>(), logp.mutable_data_ptr<float>(), seed, offset,
            static_cast<uint8_t*>(mask_out.mutable_data_ptr()), i.const_data_ptr<int64_t>(),
            i_out.mutable_data_ptr<int64_t>(), first ? first->const_data_ptr<int64_t>() : nullptr,
            first_out.mutable_data_ptr<int64_t>(), (int)take,
            static_cast<uint8_t*>(done.mutable_data_ptr()),
            static_cast<uint8_t*>(reward.mutable_data_ptr()), nullptr,
            status.mutable_data_ptr<int32_t>(), stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);  // the caller raises _native's error
    return wrap_all({&act, &logp, &mask_out, &i_out, &first_out, &done, &reward});
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// decode_step(fn, logits, mask, action_in, status, clip, temp, mode, seed, offset, full)
//   -> (act, logp, full_logprobs | None) | None
// fn: address of co_decode_step (utils/decoding.py:decode_step without top-k / top-p)
PyObject* decode_step(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 11) {
    PyErr_SetString(PyExc_TypeError, "decode_step: 11 arguments");
    return nullptr;
  }
  if (!is_tensor(a[1])) Py_RETURN_NONE;
  const auto fn = fn_at<DecodeStep>(a[0]);
  const at::Tensor& logits = THPVariable_Unpack(a[1]);
  const double clip = PyFloat_AsDouble(a[5]), temp = PyFloat_AsDouble(a[6]);
  const long mode = PyLong_AsLong(a[7]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[8]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[9]);
  const int want_full = PyObject_IsTrue(a[10]);
  if (PyErr_Occurred()) return nullptr;
  const c10::Device dev = logits.device();
  if (!dev.is_cuda() || logits.scalar_type() != at::kFloat || logits.dim() != 2 ||
      logits.stride(1) != 1)
    Py_RETURN_NONE;
  const int64_t b = logits.size(0), nl = logits.size(1);
  const at::Tensor *mask = nullptr, *ain = nullptr, *status = nullptr;
  if (is_tensor(a[2])) {
    mask = &THPVariable_Unpack(a[2]);
    if (!fits(*mask, dev, at::kBool, b * nl) || mask->dim() != 2) Py_RETURN_NONE;
  } else if (a[2] != Py_None) {
    Py_RETURN_NONE;
  }
  if (is_tensor(a[3])) {
    ain = &THPVariable_Unpack(a[3]);
    if (!fits(*ain, dev, at::kLong, b)) Py_RETURN_NONE;
  } else if (a[3] != Py_None) {
    Py_RETURN_NONE;
  }
  if (is_tensor(a[4])) {
    status = &THPVariable_Unpack(a[4]);
    if (!fits(*status, dev, at::kInt)) Py_RETURN_NONE;
  } else if (a[4] != Py_None) {
    Py_RETURN_NONE;
  }
  try {
    Carve k;
    k.chunk = at::empty({carve_bytes({8 * b, 4 * b})}, logits.options().dtype(at::kByte));
    at::Tensor act = k.take({b}, at::kLong), logp = k.take({b}, at::kFloat), full;
    if (want_full) full = at::empty({b, nl}, logits.options());
    void* stream = current_stream(dev);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, nl, logits.const_data_ptr<float>(), logits.stride(0),
            mask ? static_cast<const uint8_t*>(mask->const_data_ptr()) : nullptr, (float)clip,
            (float)temp, (int)mode, ain ? ain->const_data_ptr<int64_t>() : nullptr,
            act.mutable_data_ptr<int64_t>(), logp.mutable_data_ptr<float>(),
            want_full ? full.mutable_data_ptr<float>() : nullptr, seed, offset,
            status ? status->mutable_data_ptr<int32_t>() : nullptr, stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    return wrap_all({&act, &logp, &full});
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// cvrp_step(fn, action, demand, used, vehicle_capacity, visited)
//   -> (used_out, visited_out, current_node, done, reward, action_mask) | None
// fn: address of co_cvrp_step (envs/cvrp.py:_step)
PyObject* cvrp_step(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 6) {
    PyErr_SetString(PyExc_TypeError, "cvrp_step: 6 arguments");
    return nullptr;
  }
  for (int k = 1; k < 6; ++k)
    if (!is_tensor(a[k])) Py_RETURN_NONE;
  const auto fn = fn_at<CvrpStep>(a[0]);
  if (PyErr_Occurred()) return nullptr;
  const at::Tensor& action = THPVariable_Unpack(a[1]);
  const at::Tensor& demand = THPVariable_Unpack(a[2]);
  const at::Tensor& used = THPVariable_Unpack(a[3]);
  const at::Tensor& vcap = THPVariable_Unpack(a[4]);
  const at::Tensor& visited = THPVariable_Unpack(a[5]);
  const c10::Device dev = demand.device();
  if (!dev.is_cuda() || demand.dim() != 2) Py_RETURN_NONE;
  const int64_t b = demand.size(0), nl = demand.size(1);
  if (!fits(demand, dev, at::kFloat) || !fits(action, dev, at::kLong, b) ||
      !fits(used, dev, at::kFloat, b) || !fits(vcap, dev, at::kFloat, b) ||
      !fits(visited, dev, at::kByte, b * (nl + 1)))
    Py_RETURN_NONE;
  try {
    Carve c;
    c.chunk = at::empty({carve_bytes({4 * b, b * (nl + 1), 8 * b, b, b, b * (nl + 1)})},
                        demand.options().dtype(at::kByte));
    at::Tensor used_out = c.take(used.sizes(), at::kFloat);
    at::Tensor visited_out = c.take(visited.sizes(), at::kByte);
    at::Tensor cur = c.take({b, 1}, at::kLong), done = c.take({b}, at::kBool);
    at::Tensor reward = c.take({b}, at::kBool), mask = c.take({b, nl + 1}, at::kBool);
    void* stream = current_stream(dev);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, nl, action.const_data_ptr<int64_t>(), demand.const_data_ptr<float>(),
            used.const_data_ptr<float>(), used_out.mutable_data_ptr<float>(),
            vcap.const_data_ptr<float>(), visited.const_data_ptr<uint8_t>(),
            visited_out.mutable_data_ptr<uint8_t>(), cur.mutable_data_ptr<int64_t>(),
            static_cast<uint8_t*>(done.mutable_data_ptr()),
            static_cast<uint8_t*>(reward.mutable_data_ptr()),
            static_cast<uint8_t*>(mask.mutable_data_ptr()), nullptr, nullptr, stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    return wrap_all({&used_out, &visited_out, &cur, &done, &reward, &mask});
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyMethodDef methods[] = {
    {"decode_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(decode_step)),
     METH_FASTCALL, "decode step: outputs allocated and launched in one call"},
    {"cvrp_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(cvrp_step)),
     METH_FASTCALL, "CVRP env step: outputs allocated and launched in one call"},
    {"tsp_decode_step",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(tsp_decode_step)),
     METH_FASTCALL, "fused TSP decode step: outputs allocated and launched in one call"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_co_torchstep",
                      "drop-in decode loop host glue over the co_env C ABI", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__co_torchstep(void) { return PyModule_Create(&module); }
