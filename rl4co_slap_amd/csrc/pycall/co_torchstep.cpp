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
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "co_env.h"

namespace {

using TspDecodeStep = decltype(&co_tsp_decode_step);
using SlapDecodeStep = decltype(&co_slap_decode_step);
using CvrpDecodeStep = decltype(&co_cvrp_decode_step);
using DecodeStep = decltype(&co_decode_step);
using CvrpStep = decltype(&co_cvrp_step);
using SlapReset = decltype(&co_slap_reset);
using EpisodeStack = decltype(&co_episode_stack);

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

// Output memory.  Every output is a fresh, contiguous, non-overlapping region, 256-byte
// aligned as the caching allocator's blocks are (so the kernels' vector paths apply), made
// as a TensorImpl over a shared storage without a dispatcher call:
// * the env state of a step (mask, i, first node, done, reward; CVRP used capacity,
//   visited, current node, mask) shares one storage taken from a small per-device pool,
//   reused only when no tensor refers to it any more (storage use count 1: the pool's);
//   kernels queued on the same stream as every earlier user, as the caching allocator's
//   own reuse is;
// * the decoding strategy keeps every step's action and log-probability, so those come
//   from a slab that serves several steps (freed when its last step's tensors go).
constexpr int64_t kAlign = 256;

inline int64_t up(int64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

at::Tensor view_of(const c10::Storage& st, at::ScalarType dt, int64_t off_bytes,
                   at::IntArrayRef sizes) {
  auto impl = c10::make_intrusive<c10::TensorImpl>(
      c10::Storage(st), c10::DispatchKeySet(c10::DispatchKey::CUDA),
      c10::scalarTypeToTypeMeta(dt));
  impl->set_sizes_contiguous(sizes);
  impl->set_storage_offset(off_bytes / (int64_t)c10::elementSize(dt));
  return at::Tensor(std::move(impl));
}

// t[:, 1:] of a 2-D tensor without a dispatcher call (at::slice costs ~1 us of host time
// per step): a TensorImpl over the same storage, one element further, that shares t's
// version counter -- as a view does, so an in-place write through either is seen by the
// other's version (the env's host-side records on to_choose stay sound).
at::Tensor drop_first_col(const at::Tensor& t) {
  auto impl = c10::make_intrusive<c10::TensorImpl>(
      c10::Storage(t.storage()), c10::DispatchKeySet(c10::DispatchKey::CUDA), t.dtype());
  const int64_t sizes[2] = {t.size(0), t.size(1) - 1}, strides[2] = {t.stride(0), t.stride(1)};
  impl->set_sizes_and_strides(c10::IntArrayRef(sizes, 2), c10::IntArrayRef(strides, 2));
  impl->set_storage_offset(t.storage_offset() + t.stride(1));
  impl->set_version_counter(t.unsafeGetTensorImpl()->version_counter());
  return at::Tensor(std::move(impl));
}

c10::Storage new_storage(const c10::Device& dev, int64_t nbytes) {
  return at::empty({nbytes}, at::TensorOptions().dtype(at::kByte).device(dev)).storage();
}

// Reuse is keyed by (device, size, stream): a storage is handed out again only on the
// stream its previous users' kernels were queued on (then stream order protects them, as
// the caching allocator's own same-stream reuse does); on another stream a new storage is
// allocated.  The pool holds at most kMax storages over all keys: a new key evicts the
// least recently used free entry, so batch-size / N changes (a last partial batch, a
// validation batch) do not accumulate memory out of torch.cuda.empty_cache's reach;
// clear_pool() drops everything.
struct StatePool {
  static constexpr int kPerKey = 4, kMax = 16;
  struct Entry {
    c10::Device dev;
    int64_t nbytes;
    void* stream;
    c10::Storage st;
    uint64_t last;
  };
  std::vector<Entry> entries;
  uint64_t tick = 0;
  c10::Storage acquire(const c10::Device& dev, int64_t nbytes, void* stream) {
    ++tick;
    int same = 0;
    for (auto& e : entries) {
      if (e.dev != dev || e.nbytes != nbytes || e.stream != stream) continue;
      ++same;
      if (e.st.use_count() == 1) {
        e.last = tick;
        return e.st;
      }
    }
    c10::Storage st = new_storage(dev, nbytes);
    if (same < kPerKey) {
      if ((int)entries.size() >= kMax) evict_lru();
      if ((int)entries.size() < kMax) entries.push_back(Entry{dev, nbytes, stream, st, tick});
    }
    return st;
  }
  void evict_lru() {  // the least recently used entry nobody else refers to
    int victim = -1;
    for (int k = 0; k < (int)entries.size(); ++k)
      if (entries[k].st.use_count() == 1 && (victim < 0 || entries[k].last < entries[victim].last))
        victim = k;
    if (victim >= 0) entries.erase(entries.begin() + victim);
  }
  void clear() { entries.clear(); }
};

// The per-step [B] action and log-probability of consecutive steps are consecutive rows
// of one storage: step k takes [action row | log-probability row], so the rows of an
// episode form two step-major slabs with a uniform row stride, which the epilogue
// (episode_stack -> co_episode_stack) transposes in one launch instead of two
// torch.stack calls.  slab_fresh(steps) makes the next take start a new storage sized for
// an episode of that many steps, so an episode does not straddle two storages.
// The slab remembers the stream its rows were last handed out on: rewriting it from the
// top is safe only in that stream's order (kernels that read the last episode's rows --
// the epilogue, a reward, a caller's own launch -- were queued there), so an episode start
// on another stream takes a new storage, as StatePool::acquire does.
struct Slab {
  static constexpr int64_t kSteps = 64;
  c10::Device dev{c10::DeviceType::CPU};
  c10::Storage st;
  void* stream = nullptr;
  int64_t off = 0, cap = 0, fresh_steps = 0;
  // a region of nbytes (a multiple of kAlign) for a launch on stream s: offset into `st`
  int64_t take(const c10::Device& d, int64_t nbytes, void* s) {
    if (fresh_steps > 0 && st && d == dev && s == stream && st.use_count() == 1 &&
        nbytes * fresh_steps <= (int64_t)st.nbytes()) {
      // an episode start on a slab nothing refers to any more (the last episode's row
      // views are gone), on the stream that used it: rewrite it from the top, in stream
      // order, instead of allocating
      cap = (int64_t)st.nbytes();
      fresh_steps = 0;
      off = 0;
    } else if (!st || d != dev || off + nbytes > cap || fresh_steps > 0) {
      cap = nbytes * (fresh_steps > 0 ? fresh_steps : kSteps);
      fresh_steps = 0;
      st = new_storage(d, cap);
      dev = d;
      off = 0;
    }
    stream = s;
    const int64_t o = off;
    off += nbytes;
    return o;
  }
};

StatePool g_state;  // the GIL serialises every call into this module
Slab g_slab;

// carves one storage: take(bytes) returns the next aligned offset
struct Carver {
  int64_t off = 0;
  int64_t take(int64_t nbytes) {
    const int64_t o = off;
    off += up(nbytes);
    return o;
  }
};

// The fused TSP decode step's operand checks, output memory and launch (shared by
// tsp_decode_step and tsp_step_td).  Returns -1 when the operands do not fit (the caller's
// Python path handles them), else the C ABI's status; out = act, logp, mask_out, i_out,
// first_out, done, reward.
int tsp_launch(TspDecodeStep fn, const at::Tensor& logits, const at::Tensor& mask,
               const at::Tensor& i, const at::Tensor* first, const at::Tensor* ain,
               const at::Tensor& status, double clip, double temp, long mode, uint64_t seed,
               uint64_t offset, long take, at::Tensor (&out)[7]) {
  // the conditions envs/tsp.py:decode_and_step checks before its launch
  const c10::Device dev = mask.device();
  if (!dev.is_cuda() || logits.device() != dev || i.device() != dev || status.device() != dev ||
      logits.scalar_type() != at::kFloat || logits.dim() != 2 || logits.stride(1) != 1 ||
      mask.dim() != 2 || mask.scalar_type() != at::kBool || !mask.is_contiguous() ||
      i.scalar_type() != at::kLong || !i.is_contiguous() || status.scalar_type() != at::kInt)
    return -1;
  const int64_t b = mask.size(0), nl = mask.size(1);
  if (logits.size(0) != b || logits.size(1) != nl || nl > 2048 || i.numel() != b) return -1;
  if (!take && (!first || !fits(*first, dev, at::kLong, b))) return -1;
  if (ain && !fits(*ain, dev, at::kLong, b)) return -1;
  const int64_t kb = up(8 * b);
  void* stream = current_stream(dev);
  const int64_t ko = g_slab.take(dev, 2 * kb, stream);
  out[0] = view_of(g_slab.st, at::kLong, ko, {b});
  out[1] = view_of(g_slab.st, at::kFloat, ko + kb, {b});
  Carver c;
  const int64_t om = c.take(b * nl), oi = c.take(8 * b), of = c.take(8 * b), od = c.take(b),
                orw = c.take(b);
  const c10::Storage st = g_state.acquire(dev, c.off, stream);
  out[2] = view_of(st, at::kBool, om, {b, nl});
  out[3] = view_of(st, at::kLong, oi, i.sizes());
  out[4] = view_of(st, at::kLong, of, {b});
  out[5] = view_of(st, at::kBool, od, {b});
  out[6] = view_of(st, at::kBool, orw, {b});
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = fn(b, nl, logits.const_data_ptr<float>(), logits.stride(0),
          static_cast<const uint8_t*>(mask.const_data_ptr()), (float)clip, (float)temp, (int)mode,
          ain ? ain->const_data_ptr<int64_t>() : nullptr, out[0].mutable_data_ptr<int64_t>(),
          out[1].mutable_data_ptr<float>(), seed, offset,
          static_cast<uint8_t*>(out[2].mutable_data_ptr()), i.const_data_ptr<int64_t>(),
          out[3].mutable_data_ptr<int64_t>(), take ? nullptr : first->const_data_ptr<int64_t>(),
          out[4].mutable_data_ptr<int64_t>(), (int)take,
          static_cast<uint8_t*>(out[5].mutable_data_ptr()),
          static_cast<uint8_t*>(out[6].mutable_data_ptr()), nullptr,
          status.mutable_data_ptr<int32_t>(), stream);
  Py_END_ALLOW_THREADS
  return rc;
}

// tsp_decode_step(fn, logits, mask, i, first_in, action_in, status, clip, temp, mode,
//                 seed, offset, take) -> (act, logp, mask_out, i_out, first_out, done,
//                 reward) | None | error code
// fn: address of co_tsp_decode_step; first_in / action_in: tensor or None.
PyObject* tsp_decode_step(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 13) {
    PyErr_SetString(PyExc_TypeError, "tsp_decode_step: 13 arguments");
    return nullptr;
  }
  if (!is_tensor(a[1]) || !is_tensor(a[2]) || !is_tensor(a[3]) || !is_tensor(a[6]) ||
      (a[4] != Py_None && !is_tensor(a[4])) || (a[5] != Py_None && !is_tensor(a[5])))
    Py_RETURN_NONE;
  const auto fn = fn_at<TspDecodeStep>(a[0]);
  const double clip = PyFloat_AsDouble(a[7]), temp = PyFloat_AsDouble(a[8]);
  const long mode = PyLong_AsLong(a[9]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[10]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[11]);
  const long take = PyLong_AsLong(a[12]);
  if (PyErr_Occurred()) return nullptr;
  try {
    at::Tensor out[7];
    const int rc = tsp_launch(fn, THPVariable_Unpack(a[1]), THPVariable_Unpack(a[2]),
                              THPVariable_Unpack(a[3]),
                              is_tensor(a[4]) ? &THPVariable_Unpack(a[4]) : nullptr,
                              is_tensor(a[5]) ? &THPVariable_Unpack(a[5]) : nullptr,
                              THPVariable_Unpack(a[6]), clip, temp, mode, seed, offset, take, out);
    if (rc < 0) Py_RETURN_NONE;
    if (rc != CO_OK) return PyLong_FromLong(rc);  // the caller raises _native's error
    return wrap_all({&out[0], &out[1], &out[2], &out[3], &out[4], &out[5], &out[6]});
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// The td's keys as interned strings, made once per string literal (the literal's address
// keys the table; every caller passes a literal): a dict lookup by an interned key skips
// PyDict_GetItemString's string construction and hashing.
inline PyObject* key_of(const char* s) {
  static std::unordered_map<const char*, PyObject*> keys;
  auto it = keys.find(s);
  if (it != keys.end()) return it->second;
  PyObject* o = PyUnicode_InternFromString(s);  // kept for the process's life
  keys.emplace(s, o);
  return o;
}

// ---- host-side knowledge on state tensors (envs/base.py) ---------------------------
// A record in a tensor's instance dict, one int (version << 32) | value: valid while the
// tensor's version counter is unchanged (nobody modified it in place since the env
// produced it).  Read and written straight in the instance dict (no attribute lookup
// through the type, no tuple), a few tens of ns each.
PyObject* g_attr_i = nullptr;  // "_co_i": the value every entry of an `i` tensor holds
PyObject* g_attr_tc = nullptr;  // "_co_tc": to_choose is the env's untouched arange from k on

// the record's value, or -1 (absent / stale)
long long known(PyObject* t, PyObject* attr) {
  PyObject** dp = _PyObject_GetDictPtr(t);
  if (!dp || !*dp) return -1;
  PyObject* rec = PyDict_GetItemWithError(*dp, attr);  // borrowed
  if (!rec || !PyLong_CheckExact(rec)) {
    PyErr_Clear();
    return -1;
  }
  int overflow = 0;
  const long long r = PyLong_AsLongLongAndOverflow(rec, &overflow);
  if (overflow || r < 0) {
    PyErr_Clear();
    return -1;
  }
  if ((r >> 32) != (long long)THPVariable_Unpack(t)._version()) return -1;
  return r & 0xffffffffLL;
}

int remember(PyObject* t, PyObject* attr, long long value) {
  PyObject** dp = _PyObject_GetDictPtr(t);
  if (!dp) return PyObject_SetAttr(t, attr, Py_None);  // raises the type's error
  if (!*dp && !(*dp = PyDict_New())) return -1;
  const long long ver = (long long)THPVariable_Unpack(t)._version();
  PyObject* rec = PyLong_FromLongLong((ver << 32) | (value & 0xffffffffLL));
  if (!rec) return -1;
  const int r = PyDict_SetItem(*dp, attr, rec);
  Py_DECREF(rec);
  return r;
}

// tsp_step_td(fn, lb_attr, td, logits, mode, temp, clip, action_in, seed, offset, status,
//             key) -> (action, logp) | None | error code
// TSPEnv.decode_and_step on a dict-backed TensorDict: reads action_mask / i / first_node,
// checks the env's knowledge of i (the batch-wide first-node test), launches, records
// i + 1 and the done lower bound (attribute lb_attr) on the new state tensors and stores
// the new state in the td -- what envs/tsp.py does around tsp_decode_step, without the
// Python frames.  (fn, lb_attr) lead so that a functools.partial binds them.
PyObject* tsp_step_td(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 12) {
    PyErr_SetString(PyExc_TypeError, "tsp_step_td: 12 arguments");
    return nullptr;
  }
  PyObject* td = a[2];
  PyObject* lb_attr = a[1];
  PyObject* key = a[11];
  PyObject* ain_o = a[7];
  if (!PyDict_Check(td) || !is_tensor(a[3]) || !is_tensor(a[10]) ||
      (ain_o != Py_None && !is_tensor(ain_o)) || !PyUnicode_Check(key) ||
      !PyUnicode_Check(lb_attr))
    Py_RETURN_NONE;
  PyObject* mask_o = PyDict_GetItem(td, key_of("action_mask"));  // borrowed
  PyObject* i_o = PyDict_GetItem(td, key_of("i"));
  if (!mask_o || !i_o || !is_tensor(mask_o) || !is_tensor(i_o)) Py_RETURN_NONE;
  const long long k = known(i_o, g_attr_i);
  if (k < 0) Py_RETURN_NONE;
  const long take = k == 0 ? 1 : 0;
  PyObject* first_o = take ? nullptr : PyDict_GetItem(td, key_of("first_node"));
  if (!take && (!first_o || !is_tensor(first_o))) Py_RETURN_NONE;
  const auto fn = fn_at<TspDecodeStep>(a[0]);
  const long mode = PyLong_AsLong(a[4]);
  const double temp = PyFloat_AsDouble(a[5]), clip = PyFloat_AsDouble(a[6]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[8]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[9]);
  if (PyErr_Occurred()) return nullptr;
  at::Tensor out[7];
  try {
    const int rc = tsp_launch(fn, THPVariable_Unpack(a[3]), THPVariable_Unpack(mask_o),
                              THPVariable_Unpack(i_o),
                              first_o ? &THPVariable_Unpack(first_o) : nullptr,
                              ain_o != Py_None ? &THPVariable_Unpack(ain_o) : nullptr,
                              THPVariable_Unpack(a[10]), clip, temp, mode, seed, offset, take,
                              out);
    if (rc < 0) Py_RETURN_NONE;
    if (rc != CO_OK) return PyLong_FromLong(rc);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
  const long long lb = known(mask_o, lb_attr);
  PyObject* o[7];
  for (int j = 0; j < 7; ++j) {
    o[j] = THPVariable_Wrap(std::move(out[j]));
    if (!o[j]) {
      for (int q = 0; q < j; ++q) Py_DECREF(o[q]);
      return nullptr;
    }
  }
  PyObject* sel = ain_o != Py_None ? ain_o : o[0];
  int err = remember(o[3], g_attr_i, k + 1);
  if (!err && lb >= 0) err = remember(o[2], lb_attr, lb > 0 ? lb - 1 : 0);
  if (!err) err = PyDict_SetItem(td, key, sel);
  if (!err) err = PyDict_SetItem(td, key_of("first_node"), o[4]);
  if (!err) err = PyDict_SetItem(td, key_of("current_node"), sel);
  if (!err) err = PyDict_SetItem(td, key_of("i"), o[3]);
  if (!err) err = PyDict_SetItem(td, key_of("action_mask"), o[2]);
  if (!err) err = PyDict_SetItem(td, key_of("reward"), o[6]);
  if (!err) err = PyDict_SetItem(td, key_of("done"), o[5]);
  PyObject* res = err ? nullptr : PyTuple_Pack(2, sel, o[1]);
  for (int j = 0; j < 7; ++j) Py_DECREF(o[j]);
  return res;
}

// Wraps the 7 outputs, records i / lb, stores the new state in the td; shared tail of the
// env step_td functions.  `extra` = (key, tensor) pairs to set besides the action key.
PyObject* td_finish(PyObject* td, PyObject* key, PyObject* ain_o, at::Tensor& act,
                    at::Tensor& logp, std::initializer_list<std::pair<const char*, at::Tensor*>> st,
                    std::initializer_list<std::pair<const char*, PyObject*>> views,
                    PyObject* lb_src, PyObject* lb_attr, const char* lb_dst) {
  const long long lb = lb_src ? known(lb_src, lb_attr) : -1;
  PyObject* a_o = THPVariable_Wrap(std::move(act));
  PyObject* l_o = THPVariable_Wrap(std::move(logp));
  if (!a_o || !l_o) {
    Py_XDECREF(a_o);
    Py_XDECREF(l_o);
    return nullptr;
  }
  PyObject* sel = ain_o != Py_None ? ain_o : a_o;
  int err = PyDict_SetItem(td, key, sel);
  for (auto& kv : st) {
    if (err) break;
    PyObject* o = THPVariable_Wrap(std::move(*kv.second));
    if (!o) {
      err = -1;
      break;
    }
    if (lb >= 0 && lb_dst && std::strcmp(kv.first, lb_dst) == 0)
      err = remember(o, lb_attr, lb > 0 ? lb - 1 : 0);
    if (!err) err = PyDict_SetItem(td, key_of(kv.first), o);
    Py_DECREF(o);
  }
  for (auto& kv : views) {
    if (err) break;
    err = PyDict_SetItem(td, key_of(kv.first), kv.second);
  }
  PyObject* res = err ? nullptr : PyTuple_Pack(2, sel, l_o);
  Py_DECREF(a_o);
  Py_DECREF(l_o);
  return res;
}

inline PyObject* td_tensor(PyObject* td, const char* k) {  // borrowed; nullptr if absent
  PyObject* o = PyDict_GetItem(td, key_of(k));
  return (o && is_tensor(o)) ? o : nullptr;
}

// td[k] = a new Python object of t (the tensor moved into it); -1 on error
inline int set_wrapped(PyObject* td, const char* k, at::Tensor& t) {
  PyObject* o = THPVariable_Wrap(std::move(t));
  if (!o) return -1;
  const int err = PyDict_SetItem(td, key_of(k), o);
  Py_DECREF(o);
  return err;
}

// True when `o` (a tensor the td dict holds) is referenced by nothing but that dict: one
// Python reference, one at::Tensor handle, a storage of its own (no views, no pool), no
// autograd.  Writing it in place then cannot be told apart from writing a fresh copy.
// The reference-count test is CPython behaviour this module was built and tested on
// (3.10, with the GIL): a free-threaded build defers and biases reference counts, and
// immortal objects (3.12+) report fixed counts, so there the in-place writes are off at
// compile time and every step takes fresh storages.  CO_NO_INPLACE=1 (read at import) or
// set_inplace(False) turns them off at run time.
#if defined(Py_GIL_DISABLED) || PY_VERSION_HEX >= 0x030C0000
constexpr bool kInplaceBuild = false;
#else
constexpr bool kInplaceBuild = true;
#endif
bool g_inplace = kInplaceBuild;
// the stream of the last slap_reset_td / slap_step_td launch (none yet: a value no stream has)
void* g_slap_stream = reinterpret_cast<void*>(~uintptr_t(0));

inline bool exclusively_held(PyObject* o, const at::Tensor& t) {
  return g_inplace && Py_REFCNT(o) == 1 && t.use_count() == 1 && t.storage().use_count() == 1 &&
         !t.requires_grad() && t.is_contiguous() && t.storage_offset() == 0;
}

// The SLAP step's state block: action_mask [B, L], i [B, 1], done [B, 1], reward [B, 1]
// carved from one storage of their own (not pooled).  When the td holds the block a
// previous step made and nothing else refers to any of it -- one Python reference and one
// at::Tensor handle per tensor, the storage referenced by exactly these four -- the next
// step rewrites it in place: indistinguishable from fresh outputs (nothing can observe the
// old values), and a step then makes two tensors (action, log-probability) instead of
// six.  Otherwise a new block is carved.
struct SlapBlock {
  int64_t om, oi, od, orw, nbytes;
  SlapBlock(int64_t b, int64_t l) {
    Carver c;
    om = c.take(b * l);
    oi = c.take(8 * b);
    od = c.take(b);
    orw = c.take(b);
    nbytes = c.off;
  }
  bool held_alone(PyObject* const (&o)[4], const at::Tensor* const (&t)[4], int64_t b,
                  int64_t l) const {
    if (!g_inplace) return false;
    const c10::StorageImpl* sti = t[0]->storage().unsafeGetStorageImpl();
    if (t[0]->storage().use_count() != 4 || t[0]->storage().nbytes() != (size_t)nbytes) return false;
    const int64_t offs[4] = {om, oi / 8, od, orw};
    const at::ScalarType dts[4] = {at::kBool, at::kLong, at::kBool, at::kBool};
    for (int k = 0; k < 4; ++k) {
      const at::Tensor& x = *t[k];
      if (Py_REFCNT(o[k]) != 1 || x.use_count() != 1 || x.requires_grad() ||
          x.storage().unsafeGetStorageImpl() != sti || x.scalar_type() != dts[k] ||
          x.storage_offset() != offs[k] || !x.is_contiguous() || x.dim() != 2 || x.size(0) != b ||
          x.size(1) != (k == 0 ? l : 1))
        return false;
    }
    return true;
  }
};

// slap_step_td(fn, lb_attr, td, logits, mode, temp, clip, action_in, seed, offset, status,
//              key) -> (action, logp) | None | error code
// SLAPEnv.decode_and_step (envs/slap.py) on a dict-backed TensorDict in one call: reads
// action_mask / i / to_choose / assignment / freq, launches co_slap_decode_step, stores
// assignment / to_choose[:, 1:] / action_mask / i / reward / done and the action, records
// the done lower bound on the new i.  Savings invisible to the caller:
// * to_choose that is still the env's untouched arange (record "_co_tc" = k, version
//   unchanged) is not read: the kernel takes the uniform product k (co_env.h);
// * the assignment is the reference's clone with one element changed (slap/env.py:50-54):
//   when nothing but the td refers to the input assignment, that element is written in
//   place; otherwise the row is copied into a new storage of its own (so the next step can
//   write it in place);
// * the state block (SlapBlock) likewise: in place when held by the td alone.
PyObject* slap_step_td(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 12) {
    PyErr_SetString(PyExc_TypeError, "slap_step_td: 12 arguments");
    return nullptr;
  }
  PyObject* lb_attr = a[1];
  PyObject* td = a[2];
  PyObject* key = a[11];
  PyObject* ain_o = a[7];
  if (!PyDict_Check(td) || !is_tensor(a[3]) || !is_tensor(a[10]) ||
      (ain_o != Py_None && !is_tensor(ain_o)) || !PyUnicode_Check(key) || !PyUnicode_Check(lb_attr))
    Py_RETURN_NONE;
  PyObject *mask_o = td_tensor(td, "action_mask"), *i_o = td_tensor(td, "i"),
           *tc_o = td_tensor(td, "to_choose"), *as_o = td_tensor(td, "assignment"),
           *fr_o = td_tensor(td, "freq"), *dn_o = td_tensor(td, "done"),
           *rw_o = td_tensor(td, "reward");
  if (!mask_o || !i_o || !tc_o || !as_o || !fr_o) Py_RETURN_NONE;
  const auto fn = fn_at<SlapDecodeStep>(a[0]);
  const long long ki = known(i_o, g_attr_i);
  const long long ktc = known(tc_o, g_attr_tc);
  const long long lb = known(i_o, lb_attr);
  const long mode = PyLong_AsLong(a[4]);
  const double temp = PyFloat_AsDouble(a[5]), clip = PyFloat_AsDouble(a[6]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[8]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[9]);
  if (PyErr_Occurred()) return nullptr;
  try {
    const at::Tensor& logits = THPVariable_Unpack(a[3]);
    const at::Tensor& mask = THPVariable_Unpack(mask_o);
    const at::Tensor& i = THPVariable_Unpack(i_o);
    const at::Tensor& tc = THPVariable_Unpack(tc_o);
    const at::Tensor& asg = THPVariable_Unpack(as_o);
    const at::Tensor& status = THPVariable_Unpack(a[10]);
    const at::Tensor* ain = ain_o != Py_None ? &THPVariable_Unpack(ain_o) : nullptr;
    const c10::Device dev = mask.device();
    // the conditions envs/slap.py:decode_and_step checks
    if (!dev.is_cuda() || logits.device() != dev || logits.scalar_type() != at::kFloat ||
        logits.dim() != 2 || logits.stride(1) != 1 || mask.dim() != 2 ||
        mask.scalar_type() != at::kBool || !mask.is_contiguous() || tc.dim() != 2 ||
        tc.device() != dev || tc.scalar_type() != at::kFloat || tc.stride(1) != 1 ||
        tc.size(1) < 1 || status.device() != dev || status.scalar_type() != at::kInt)
      Py_RETURN_NONE;
    const at::Tensor& fr = THPVariable_Unpack(fr_o);
    const int64_t b = mask.size(0), l = mask.size(1);
    if (fr.dim() < 2) Py_RETURN_NONE;
    const int64_t p = fr.size(fr.dim() - 2);
    if (logits.size(0) != b || logits.size(1) != l || l > 2048 || tc.size(0) != b ||
        !fits(i, dev, at::kLong, b) || !fits(asg, dev, at::kInt, b * p) || asg.dim() != 2 ||
        asg.size(0) != b)
      Py_RETURN_NONE;
    if (ain && !fits(*ain, dev, at::kLong, b)) Py_RETURN_NONE;
    // the untouched arange: to_choose[:, 0] == k in every row (k + remaining columns == P)
    const bool uniform = ktc >= 0 && ktc < p && ktc + tc.size(1) == p;
    void* stream = current_stream(dev);
    // in place only in the stream order of the previous step's launch (which made the
    // tensors or last read them)
    const bool same_stream = stream == g_slap_stream;
    g_slap_stream = stream;
    const bool asg_here = same_stream && exclusively_held(as_o, asg);
    const SlapBlock blk(b, l);
    bool blk_here = false;
    if (same_stream && dn_o && rw_o) {
      PyObject* const os[4] = {mask_o, i_o, dn_o, rw_o};
      const at::Tensor* const ts[4] = {&mask, &i, &THPVariable_Unpack(dn_o), &THPVariable_Unpack(rw_o)};
      blk_here = blk.held_alone(os, ts, b, l);
    }
    const int64_t kb = up(8 * b);
    const int64_t ko = g_slab.take(dev, 2 * kb, stream);
    at::Tensor act = view_of(g_slab.st, at::kLong, ko, {b});
    at::Tensor logp = view_of(g_slab.st, at::kFloat, ko + kb, {b});
    at::Tensor asg_out = asg_here ? asg : view_of(new_storage(dev, 4 * b * p), at::kInt, 0,
                                                  asg.sizes());
    at::Tensor mask_out, i_out, done, reward;
    if (blk_here) {
      mask_out = mask;
      i_out = i;
      done = THPVariable_Unpack(dn_o);
      reward = THPVariable_Unpack(rw_o);
    } else {
      const c10::Storage st = new_storage(dev, blk.nbytes);
      mask_out = view_of(st, at::kBool, blk.om, {b, l});
      i_out = view_of(st, at::kLong, blk.oi, {b, 1});
      done = view_of(st, at::kBool, blk.od, {b, 1});
      reward = view_of(st, at::kBool, blk.orw, {b, 1});
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, l, p, logits.const_data_ptr<float>(), logits.stride(0),
            static_cast<const uint8_t*>(mask.const_data_ptr()), (float)clip, (float)temp, (int)mode,
            ain ? ain->const_data_ptr<int64_t>() : nullptr, act.mutable_data_ptr<int64_t>(),
            logp.mutable_data_ptr<float>(), seed, offset,
            uniform ? nullptr : tc.const_data_ptr<float>(), uniform ? ktc : tc.stride(0),
            asg.const_data_ptr<int32_t>(), asg_out.mutable_data_ptr<int32_t>(),
            static_cast<uint8_t*>(mask_out.mutable_data_ptr()), i.const_data_ptr<int64_t>(),
            i_out.mutable_data_ptr<int64_t>(), static_cast<uint8_t*>(done.mutable_data_ptr()),
            static_cast<uint8_t*>(reward.mutable_data_ptr()), nullptr,
            status.mutable_data_ptr<int32_t>(), stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    if (asg_here) asg.unsafeGetTensorImpl()->bump_version();  // in-place writes
    if (blk_here) {
      mask.unsafeGetTensorImpl()->bump_version();
      i.unsafeGetTensorImpl()->bump_version();
      done.unsafeGetTensorImpl()->bump_version();
      reward.unsafeGetTensorImpl()->bump_version();
    }
    PyObject* tc_next = THPVariable_Wrap(drop_first_col(tc));  // to_choose[:, 1:]
    if (!tc_next) return nullptr;
    int err = uniform ? remember(tc_next, g_attr_tc, ktc + 1) : 0;
    if (!err) err = PyDict_SetItem(td, key_of("to_choose"), tc_next);
    Py_DECREF(tc_next);
    if (err) return nullptr;
    PyObject* a_o = THPVariable_Wrap(std::move(act));
    PyObject* l_o = a_o ? THPVariable_Wrap(std::move(logp)) : nullptr;
    if (!a_o || !l_o) {
      Py_XDECREF(a_o);
      return nullptr;
    }
    PyObject* sel = ain_o != Py_None ? ain_o : a_o;
    err = PyDict_SetItem(td, key, sel);
    if (!err && !asg_here) err = set_wrapped(td, "assignment", asg_out);
    if (!err && !blk_here) {
      err = set_wrapped(td, "action_mask", mask_out);
      if (!err) err = set_wrapped(td, "i", i_out);
      if (!err) err = set_wrapped(td, "reward", reward);
      if (!err) err = set_wrapped(td, "done", done);
    }
    // records on the new i / done: the done lower bound (lb - 1), and -- i uniform over the
    // batch when the env knows its value (reset: 0; each step +1) -- i + 1 and done = (i ==
    // P-1), so poll_done answers without a read
    if (!err) {
      PyObject* i_n = PyDict_GetItem(td, key_of("i"));
      PyObject* d_n = PyDict_GetItem(td, key_of("done"));
      if (!i_n || !d_n) err = -1;
      if (!err && lb >= 0) err = remember(i_n, lb_attr, lb > 0 ? lb - 1 : 0);
      if (!err && ki >= 0) {
        err = remember(i_n, g_attr_i, ki + 1);
        if (!err) err = remember(d_n, g_attr_i, ki == p - 1 ? 1 : 0);
      }
    }
    PyObject* res = err ? nullptr : PyTuple_Pack(2, sel, l_o);
    Py_DECREF(a_o);
    Py_DECREF(l_o);
    return res;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// cvrp_step_td(fn, lb_attr, td, logits, mode, temp, clip, action_in, seed, offset, status,
//              key) -> (action, logp) | None | error code
// CVRPEnv.decode_and_step (envs/cvrp.py) on a dict-backed TensorDict in one call.
PyObject* cvrp_step_td(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 12) {
    PyErr_SetString(PyExc_TypeError, "cvrp_step_td: 12 arguments");
    return nullptr;
  }
  PyObject* lb_attr = a[1];
  PyObject* td = a[2];
  PyObject* key = a[11];
  PyObject* ain_o = a[7];
  if (!PyDict_Check(td) || !is_tensor(a[3]) || !is_tensor(a[10]) ||
      (ain_o != Py_None && !is_tensor(ain_o)) || !PyUnicode_Check(key) || !PyUnicode_Check(lb_attr))
    Py_RETURN_NONE;
  PyObject *mask_o = td_tensor(td, "action_mask"), *dem_o = td_tensor(td, "demand"),
           *used_o = td_tensor(td, "used_capacity"), *cap_o = td_tensor(td, "vehicle_capacity"),
           *vis_o = td_tensor(td, "visited");
  if (!mask_o || !dem_o || !used_o || !cap_o || !vis_o) Py_RETURN_NONE;
  const auto fn = fn_at<CvrpDecodeStep>(a[0]);
  const long mode = PyLong_AsLong(a[4]);
  const double temp = PyFloat_AsDouble(a[5]), clip = PyFloat_AsDouble(a[6]);
  const uint64_t seed = PyLong_AsUnsignedLongLongMask(a[8]);
  const uint64_t offset = PyLong_AsUnsignedLongLongMask(a[9]);
  if (PyErr_Occurred()) return nullptr;
  try {
    const at::Tensor& logits = THPVariable_Unpack(a[3]);
    const at::Tensor& mask = THPVariable_Unpack(mask_o);
    const at::Tensor& dem = THPVariable_Unpack(dem_o);
    const at::Tensor& used = THPVariable_Unpack(used_o);
    const at::Tensor& cap = THPVariable_Unpack(cap_o);
    const at::Tensor& vis = THPVariable_Unpack(vis_o);
    const at::Tensor& status = THPVariable_Unpack(a[10]);
    const at::Tensor* ain = ain_o != Py_None ? &THPVariable_Unpack(ain_o) : nullptr;
    const c10::Device dev = dem.device();
    if (!dev.is_cuda() || dem.dim() != 2 || logits.device() != dev ||
        logits.scalar_type() != at::kFloat || logits.dim() != 2 || logits.stride(1) != 1 ||
        status.device() != dev || status.scalar_type() != at::kInt)
      Py_RETURN_NONE;
    const int64_t b = dem.size(0), nl = dem.size(1);
    if (logits.size(0) != b || logits.size(1) != nl + 1 || nl + 1 > 2048 ||
        !fits(dem, dev, at::kFloat) || !fits(used, dev, at::kFloat, b) ||
        !fits(cap, dev, at::kFloat, b) || !fits(vis, dev, at::kByte, b * (nl + 1)) ||
        !fits(mask, dev, at::kBool, b * (nl + 1)) || mask.dim() != 2)
      Py_RETURN_NONE;
    if (ain && !fits(*ain, dev, at::kLong, b)) Py_RETURN_NONE;
    const int64_t kb = up(8 * b);
    void* stream = current_stream(dev);
    const int64_t ko = g_slab.take(dev, 2 * kb, stream);
    at::Tensor act = view_of(g_slab.st, at::kLong, ko, {b});
    at::Tensor logp = view_of(g_slab.st, at::kFloat, ko + kb, {b});
    Carver c;
    const int64_t ou = c.take(4 * b), ov = c.take(b * (nl + 1)), oc = c.take(8 * b),
                  od = c.take(b), orw = c.take(b), om = c.take(b * (nl + 1));
    const c10::Storage st = g_state.acquire(dev, c.off, stream);
    at::Tensor used_out = view_of(st, at::kFloat, ou, used.sizes());
    at::Tensor vis_out = view_of(st, at::kByte, ov, vis.sizes());
    at::Tensor cur = view_of(st, at::kLong, oc, {b, 1});
    at::Tensor done = view_of(st, at::kBool, od, {b});
    at::Tensor reward = view_of(st, at::kBool, orw, {b});
    at::Tensor mask_out = view_of(st, at::kBool, om, {b, nl + 1});
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, nl, logits.const_data_ptr<float>(), logits.stride(0),
            static_cast<const uint8_t*>(mask.const_data_ptr()), (float)clip, (float)temp, (int)mode,
            ain ? ain->const_data_ptr<int64_t>() : nullptr, act.mutable_data_ptr<int64_t>(),
            logp.mutable_data_ptr<float>(), seed, offset, dem.const_data_ptr<float>(),
            used.const_data_ptr<float>(), used_out.mutable_data_ptr<float>(),
            cap.const_data_ptr<float>(), vis.const_data_ptr<uint8_t>(),
            vis_out.mutable_data_ptr<uint8_t>(), cur.mutable_data_ptr<int64_t>(),
            static_cast<uint8_t*>(done.mutable_data_ptr()),
            static_cast<uint8_t*>(reward.mutable_data_ptr()),
            static_cast<uint8_t*>(mask_out.mutable_data_ptr()), nullptr,
            status.mutable_data_ptr<int32_t>(), stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    return td_finish(td, key, ain_o, act, logp,
                     {{"current_node", &cur}, {"used_capacity", &used_out},
                      {"visited", &vis_out}, {"reward", &reward}, {"done", &done},
                      {"action_mask", &mask_out}},
                     {}, vis_o, lb_attr, "visited");
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
    const int64_t kb = up(8 * b);
    void* stream = current_stream(dev);
    const int64_t ko = g_slab.take(dev, 2 * kb, stream);
    at::Tensor act = view_of(g_slab.st, at::kLong, ko, {b});
    at::Tensor logp = view_of(g_slab.st, at::kFloat, ko + kb, {b}), full;
    if (want_full) full = at::empty({b, nl}, logits.options());
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
    Carver c;
    const int64_t ou = c.take(4 * b), ov = c.take(b * (nl + 1)), oc = c.take(8 * b),
                  od = c.take(b), orw = c.take(b), om = c.take(b * (nl + 1));
    void* stream = current_stream(dev);
    const c10::Storage st = g_state.acquire(dev, c.off, stream);
    at::Tensor used_out = view_of(st, at::kFloat, ou, used.sizes());
    at::Tensor visited_out = view_of(st, at::kByte, ov, visited.sizes());
    at::Tensor cur = view_of(st, at::kLong, oc, {b, 1});
    at::Tensor done = view_of(st, at::kBool, od, {b});
    at::Tensor reward = view_of(st, at::kBool, orw, {b});
    at::Tensor mask = view_of(st, at::kBool, om, {b, nl + 1});
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

// slab_fresh(steps) -> None: the next step's action / log-probability rows start a new
// slab storage sized for `steps` steps (DecodingStrategy calls it at an episode's first
// step with the env's bound on the episode length)
PyObject* slab_fresh(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 1) {
    PyErr_SetString(PyExc_TypeError, "slab_fresh: 1 argument");
    return nullptr;
  }
  const long long steps = PyLong_AsLongLong(a[0]);
  if (PyErr_Occurred()) return nullptr;
  g_slab.fresh_steps = steps < 1 ? 1 : (steps > 4096 ? 4096 : steps);
  Py_RETURN_NONE;
}

// episode_stack(fn, actions, logprobs, status, want_ll) -> (actions[B,T], logprobs[B,T],
//   ll[B] | None) | None | error code
// DecodingStrategy.post_decoder_hook's torch.stack(self.actions, 1) / torch.stack(
// self.logprobs, 1), get_log_likelihood's sum and its `> -1000` test (CO_ST_LOGP_NEG_INF in
// status) as one co_episode_stack launch -- when the two lists hold [B] tensors that are
// consecutive rows of step-major slabs (what the step calls above return); None otherwise
// (the caller stacks as before).
PyObject* episode_stack(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 5) {
    PyErr_SetString(PyExc_TypeError, "episode_stack: 5 arguments");
    return nullptr;
  }
  PyObject *al = a[1], *ll_ = a[2];
  if (!PyList_Check(al) || !PyList_Check(ll_) || !is_tensor(a[3])) Py_RETURN_NONE;
  const Py_ssize_t T = PyList_GET_SIZE(al);
  if (T < 1 || PyList_GET_SIZE(ll_) != T) Py_RETURN_NONE;
  const auto fn = fn_at<EpisodeStack>(a[0]);
  const int want_ll = PyObject_IsTrue(a[4]);
  if (want_ll < 0) return nullptr;
  try {
    const at::Tensor& status = THPVariable_Unpack(a[3]);
    // the rows: [B] tensors, one storage per list, a uniform stride between steps
    int64_t b = -1, rs[2] = {0, 0};
    const void* base[2] = {nullptr, nullptr};
    c10::Device dev{c10::DeviceType::CPU};
    for (int li = 0; li < 2; ++li) {
      PyObject* lst = li == 0 ? al : ll_;
      const at::ScalarType dt = li == 0 ? at::kLong : at::kFloat;
      const int64_t esz = li == 0 ? 8 : 4;
      const c10::StorageImpl* sti = nullptr;
      for (Py_ssize_t t = 0; t < T; ++t) {
        PyObject* o = PyList_GET_ITEM(lst, t);
        if (!is_tensor(o)) Py_RETURN_NONE;
        const at::Tensor& x = THPVariable_Unpack(o);
        if (x.dim() != 1 || x.scalar_type() != dt || x.stride(0) != 1 || x.requires_grad())
          Py_RETURN_NONE;
        if (t == 0 && li == 0) {
          dev = x.device();
          b = x.size(0);
          if (!dev.is_cuda() || b < 1) Py_RETURN_NONE;
        }
        if (x.device() != dev || x.size(0) != b) Py_RETURN_NONE;
        const char* p = static_cast<const char*>(x.const_data_ptr());
        if (t == 0) {
          base[li] = p;
          sti = x.storage().unsafeGetStorageImpl();
        } else {
          if (x.storage().unsafeGetStorageImpl() != sti) Py_RETURN_NONE;
          const int64_t d = p - static_cast<const char*>(base[li]);
          if (t == 1) {
            if (d <= 0 || d % esz != 0 || d / esz < b) Py_RETURN_NONE;
            rs[li] = d / esz;
          } else if (d != (int64_t)t * rs[li] * esz) {
            Py_RETURN_NONE;
          }
        }
      }
      if (T == 1) rs[li] = b;
    }
    if (status.device() != dev || status.scalar_type() != at::kInt) Py_RETURN_NONE;
    // the three outputs carved from one storage (one allocation instead of three)
    Carver cv;
    const int64_t oa = cv.take(8 * b * (int64_t)T), ol = cv.take(4 * b * (int64_t)T),
                  os = cv.take(4 * b);
    const c10::Storage ost = new_storage(dev, cv.off);
    at::Tensor acts = view_of(ost, at::kLong, oa, {b, (int64_t)T});
    at::Tensor lps = view_of(ost, at::kFloat, ol, {b, (int64_t)T});
    at::Tensor ll;
    if (want_ll) ll = view_of(ost, at::kFloat, os, {b});
    void* stream = current_stream(dev);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, (int64_t)T, static_cast<const int64_t*>(base[0]), rs[0],
            static_cast<const float*>(base[1]), rs[1], acts.mutable_data_ptr<int64_t>(),
            lps.mutable_data_ptr<float>(), want_ll ? ll.mutable_data_ptr<float>() : nullptr,
            status.mutable_data_ptr<int32_t>(), stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    return wrap_all({&acts, &lps, &ll});
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// slap_reset_td(fn, lb_attr, td) -> True | None | error code
// SLAPEnv._reset (slap/env.py:95-129) + RL4COEnvBase.reset's done / terminated zeros on a
// dict-backed TensorDict in one co_slap_reset launch: mask / to_choose / i / reward /
// ratio / done / terminated carved from one storage and stored in the td; records i = 0,
// the done lower bound P, and the untouched-arange record of to_choose (offset 0).
PyObject* slap_reset_td(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 3) {
    PyErr_SetString(PyExc_TypeError, "slap_reset_td: 3 arguments");
    return nullptr;
  }
  PyObject *lb_attr = a[1], *td = a[2];
  if (!PyDict_Check(td) || !PyUnicode_Check(lb_attr)) Py_RETURN_NONE;
  PyObject *as_o = td_tensor(td, "assignment"), *fr_o = td_tensor(td, "freq"),
           *lo_o = td_tensor(td, "locs"), *dd_o = td_tensor(td, "depot_loc_dist");
  if (!as_o || !fr_o || !lo_o || !dd_o) Py_RETURN_NONE;
  const auto fn = fn_at<SlapReset>(a[0]);
  try {
    const at::Tensor& asg = THPVariable_Unpack(as_o);
    const at::Tensor& fr = THPVariable_Unpack(fr_o);
    const at::Tensor& lo = THPVariable_Unpack(lo_o);
    const at::Tensor& dd = THPVariable_Unpack(dd_o);
    const c10::Device dev = asg.device();
    if (!dev.is_cuda() || asg.dim() < 1 || fr.dim() < 2 || lo.dim() < 2 || dd.dim() != 2)
      Py_RETURN_NONE;
    const int64_t b = asg.size(0), p = fr.size(fr.dim() - 2), l = lo.size(1);
    if (dd.size(0) != b || dd.size(1) != l) Py_RETURN_NONE;
    Carver c;
    const int64_t om = c.take(b * l), ot = c.take(4 * b * p), oi = c.take(8 * b),
                  orw = c.take(4 * b), ora = c.take(4 * b * l), od = c.take(b), oe = c.take(b);
    c10::Storage st = new_storage(dev, c.off);
    at::Tensor mask = view_of(st, at::kBool, om, {b, l});
    at::Tensor tc = view_of(st, at::kFloat, ot, {b, p});
    at::Tensor it = view_of(st, at::kLong, oi, {b, 1});
    at::Tensor rw = view_of(st, at::kFloat, orw, {b, 1});
    at::Tensor ratio = view_of(st, at::kFloat, ora, {b, l});
    at::Tensor done = view_of(st, at::kBool, od, {b, 1});
    at::Tensor term = view_of(st, at::kBool, oe, {b, 1});
    void* stream = current_stream(dev);
    g_slap_stream = stream;  // the episode's tensors are made in this stream's order
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(b, l, p, static_cast<uint8_t*>(mask.mutable_data_ptr()), tc.mutable_data_ptr<float>(),
            it.mutable_data_ptr<int64_t>(), rw.mutable_data_ptr<float>(),
            ratio.mutable_data_ptr<float>(), static_cast<uint8_t*>(done.mutable_data_ptr()),
            static_cast<uint8_t*>(term.mutable_data_ptr()), stream);
    Py_END_ALLOW_THREADS
    if (rc != CO_OK) return PyLong_FromLong(rc);
    std::pair<const char*, at::Tensor*> outs[] = {
        {"to_choose", &tc}, {"i", &it},       {"ratio", &ratio},   {"action_mask", &mask},
        {"reward", &rw},    {"done", &done}, {"terminated", &term}};
    for (auto& kv : outs) {
      PyObject* o = THPVariable_Wrap(std::move(*kv.second));
      if (!o) return nullptr;
      int err = 0;
      if (kv.first[0] == 'i') err = remember(o, g_attr_i, 0) || remember(o, lb_attr, p);
      else if (kv.first[0] == 't' && kv.first[1] == 'o') err = remember(o, g_attr_tc, 0);
      if (!err) err = PyDict_SetItem(td, key_of(kv.first), o);
      Py_DECREF(o);
      if (err) return nullptr;
    }
    Py_RETURN_TRUE;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// set_inplace(flag) -> previous flag: allow the in-place state writes (only where the
// build allows them: kInplaceBuild); inplace_policy() -> (build allows, enabled)
PyObject* set_inplace(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 1) {
    PyErr_SetString(PyExc_TypeError, "set_inplace: 1 argument");
    return nullptr;
  }
  const int v = PyObject_IsTrue(a[0]);
  if (v < 0) return nullptr;
  const bool prev = g_inplace;
  g_inplace = kInplaceBuild && v;
  return PyBool_FromLong(prev);
}
PyObject* inplace_policy(PyObject*, PyObject* const*, Py_ssize_t) {
  return Py_BuildValue("(OO)", kInplaceBuild ? Py_True : Py_False, g_inplace ? Py_True : Py_False);
}

// fast_step(native, td_type, mword, temp, clip, status, key, actions, logprobs, strategy,
//           idx_attr, check_rc, td, logits, mask) -> bool
// The per-step closure of DecodingStrategy.fast_stepper (utils/decoding.py) in C, bound
// with functools.partial over everything but (td, logits, mask): False, having done
// nothing, when td is not of td_type or mask is not the td's action_mask (the caller then
// takes step_env_fused); else native(td, logits, mword, temp, clip, None, 0,
// strategy.<idx_attr>, status, key) -- an env's *_step_td glue -- whose None also means
// False and whose int status goes to check_rc("decode_and_step", rc); then
// strategy.<idx_attr> += 1 and the (action, logp) pair appended to the two lists.  The
// same calls in the same order as the Python closure, without its frame per step.
PyObject* fast_step(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 15) {
    PyErr_SetString(PyExc_TypeError, "fast_step: 15 arguments");
    return nullptr;
  }
  PyObject *td = a[12], *logits = a[13], *mask = a[14];
  if (reinterpret_cast<PyObject*>(Py_TYPE(td)) != a[1] || !PyDict_Check(td) ||
      PyDict_GetItem(td, key_of("action_mask")) != mask)
    Py_RETURN_FALSE;
  if (!PyList_Check(a[7]) || !PyList_Check(a[8])) {
    PyErr_SetString(PyExc_TypeError, "fast_step: the action / log-probability lists");
    return nullptr;
  }
  PyObject* idx = PyObject_GetAttr(a[9], a[10]);
  if (!idx) return nullptr;
  PyObject* zero = PyLong_FromLong(0);
  if (!zero) {
    Py_DECREF(idx);
    return nullptr;
  }
  PyObject* args[10] = {td, logits, a[2], a[3], a[4], Py_None, zero, idx, a[5], a[6]};
  PyObject* out = PyObject_Vectorcall(a[0], args, 10, nullptr);
  Py_DECREF(zero);
  if (!out || out == Py_None) {
    Py_DECREF(idx);
    if (!out) return nullptr;
    Py_DECREF(out);
    Py_RETURN_FALSE;
  }
  if (PyLong_Check(out)) {  // an error code: check_rc raises it
    Py_DECREF(idx);
    PyObject* name = PyUnicode_FromString("decode_and_step");
    PyObject* r = nullptr;
    if (name) {
      PyObject* cargs[2] = {name, out};
      r = PyObject_Vectorcall(a[11], cargs, 2, nullptr);
      Py_DECREF(name);
    }
    Py_DECREF(out);
    if (!r) return nullptr;
    Py_DECREF(r);
    PyErr_SetString(PyExc_RuntimeError, "decode_and_step returned a status and no outputs");
    return nullptr;
  }
  if (!PyTuple_Check(out) || PyTuple_GET_SIZE(out) != 2) {
    Py_DECREF(idx);
    Py_DECREF(out);
    PyErr_SetString(PyExc_TypeError, "fast_step: the step glue returned no (action, logp)");
    return nullptr;
  }
  PyObject* one = PyLong_FromLong(1);
  PyObject* nidx = one ? PyNumber_Add(idx, one) : nullptr;
  Py_XDECREF(one);
  Py_DECREF(idx);
  int err = nidx ? PyObject_SetAttr(a[9], a[10], nidx) : -1;
  Py_XDECREF(nidx);
  if (!err) err = PyList_Append(a[7], PyTuple_GET_ITEM(out, 0));
  if (!err) err = PyList_Append(a[8], PyTuple_GET_ITEM(out, 1));
  Py_DECREF(out);
  if (err) return nullptr;
  Py_RETURN_TRUE;
}

// clear_pool() -> None: drop every pooled state storage (tensors still held stay valid)
PyObject* clear_pool(PyObject*, PyObject* const*, Py_ssize_t) {
  g_state.clear();
  Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"slap_step_td", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(slap_step_td)),
     METH_FASTCALL, "SLAPEnv.decode_and_step on a dict-backed TensorDict, in one call"},
    {"cvrp_step_td", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(cvrp_step_td)),
     METH_FASTCALL, "CVRPEnv.decode_and_step on a dict-backed TensorDict, in one call"},
    {"set_inplace", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(set_inplace)),
     METH_FASTCALL, "allow / forbid the in-place state writes; returns the previous flag"},
    {"inplace_policy",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(inplace_policy)),
     METH_FASTCALL, "(build allows in-place writes, enabled)"},
    {"fast_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(fast_step)),
     METH_FASTCALL, "the greedy decode loop's per-step closure (fast_stepper) in C"},
    {"clear_pool", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(clear_pool)),
     METH_FASTCALL, "drop the pooled step-state storages"},
    {"slab_fresh", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(slab_fresh)),
     METH_FASTCALL, "start a new action / log-probability slab at the next step"},
    {"episode_stack",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(episode_stack)),
     METH_FASTCALL, "the decode loop's stack + log-likelihood epilogue in one launch"},
    {"slap_reset_td",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(slap_reset_td)),
     METH_FASTCALL, "SLAPEnv._reset + the reset's done / terminated in one launch"},
    {"tsp_step_td", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(tsp_step_td)),
     METH_FASTCALL, "TSPEnv.decode_and_step on a dict-backed TensorDict, in one call"},
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

PyMODINIT_FUNC PyInit__co_torchstep(void) {
  g_attr_i = PyUnicode_InternFromString("_co_i");
  g_attr_tc = PyUnicode_InternFromString("_co_tc");
  if (!g_attr_i || !g_attr_tc) return nullptr;
  const char* no_inplace = std::getenv("CO_NO_INPLACE");
  if (no_inplace && no_inplace[0] && no_inplace[0] != '0') g_inplace = false;
  return PyModule_Create(&module);
}
