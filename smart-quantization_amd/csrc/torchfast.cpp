// torchfast.cpp — the eager per-call host path of SmartFP and S2FP8 in one C call, and the
// autograd wrapper of SmartFP as a C++ graph node (module _smqtorch, built next to libsmq.so and
// linked to it and to libtorch).
//
// An eager training step that compresses every layer's activation and grad-map issues one codec
// call per layer output in the forward pass and one per grad-map in the backward pass (reference:
// smart_compress/util/pytorch/autograd.py:18-47 around smart.py:110-190; bench.py --config
// autograd_resnet34: 264 calls per step). With ~8 us of device time per call the eager step is
// bound by the host time of those calls: the Python codec path spent ~6.75 us per call (output
// allocation through torch's Python binding, the parameter-block copy, the stream query, the
// workspace lookup, the offset update, the argument conversion), the Python autograd Function
// around it as much again in each direction. Here:
//
//   smaq(state, x, all_positive, bn)        one SmartFP call on the at::Tensor (smq_smaq_roundtrip;
//                                           with ratio logging smq_smaq_roundtrip_counted and
//                                           (y, values): the log_size values stay on the device)
//   smaq_autograd(state, x, codec, bwd)     Compressor.forward for a SmartFP codec: the forward
//                                           call plus a C++ Node whose backward compresses the
//                                           grad-map the same way (autograd.py:37-47)
//   smaq_packed(state, x, ap, getter, frac[, notify])  PackedActivations' forward call: y and its
//                                           SmaQ stream (smq_smaq_roundtrip_compress_notify,
//                                           util/pytorch/saved.py; notify: the address of a
//                                           host-mapped word that receives the stream's size)
//   smaq_packed_autograd(state, x, acts, bwd, getter, frac[, notify])  the same call from
//                                           Compressor.forward, y with the SmaqCompressBackward node
//   smaq_unpacked(data, shape, n, bm, bo)   its backward decode (smq_smaq_decompress_ex)
//   s2fp8(x, check_inf, rng, getter)        one S2FP8 call on an fp32 device tensor
//
// The state object (a capsule of a shared SmaqState) holds the flag templates of the parameter
// block, built by the Python codec from its hparams, and a snapshot of the hparams values they were
// built from: a flag changed between calls returns NotImplemented and the codec rebuilds the state.
// Anything this path does not handle (CPU tensors, float64, sampled or range statistics, BN terms,
// graph-safe streams, tensors below min_size) returns None and the codec takes its
// general Python path (in the backward node: the Python codec object is called). Values are those
// of the Python path bit for bit: the same entry point, parameter block and stream positions, taken
// in the same call order. Host code only; nothing here crosses the C-ABI (include/smq.h).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <ATen/ops/zeros.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/utils.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstddef>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "smq.h"

namespace {

// Python objects held by C++ objects that may die on an autograd worker thread
struct PyRef {
  PyObject* o = nullptr;
  PyRef() = default;
  explicit PyRef(PyObject* p) : o(p) { Py_XINCREF(o); }
  PyRef(const PyRef&) = delete;
  PyRef& operator=(const PyRef&) = delete;
  ~PyRef() {
    if (o && Py_IsInitialized()) {
      PyGILState_STATE g = PyGILState_Ensure();
      Py_DECREF(o);
      PyGILState_Release(g);
    }
  }
};

// The (device, stream) workspace of the last call: the Python table (smart_compress_amd/_native.py
// workspace) is asked only when the device, the stream or the needed size changes. The tensor is
// held here, so the table evicting it never frees memory a queued call still uses.
struct WsSlot {
  int dev = -1;
  hipStream_t st = nullptr;
  at::Tensor t;
  void* ptr = nullptr;
  size_t bytes = 0;
};

// Python getter(device_index, stream, nbytes) -> uint8 device tensor (the codec's _native.workspace)
bool ws_lookup(WsSlot& w, PyObject* getter, int dev, hipStream_t st, size_t need) {
  if (w.ptr && w.dev == dev && w.st == st && w.bytes >= need) return true;
  PyObject* r = PyObject_CallFunction(getter, "iKn", dev, (unsigned long long)(uintptr_t)st,
                                      (Py_ssize_t)need);
  if (!r) return false;
  if (!THPVariable_Check(r)) {
    Py_DECREF(r);
    PyErr_SetString(PyExc_TypeError, "workspace getter must return a tensor");
    return false;
  }
  w.t = THPVariable_Unpack(r);
  Py_DECREF(r);
  w.dev = dev;
  w.st = st;
  w.ptr = w.t.data_ptr();
  w.bytes = (size_t)w.t.numel();
  return true;
}

// --measure_compression_ratio: one zeroed SmqSizeRecord per call (smq_smaq_roundtrip_counted) from
// a pool per (device, stream) — one zero-fill per kPoolRecs calls, on the stream that uses the
// records. The values the logger gets are views of the record (kept alive by them).
constexpr int64_t kPoolRecs = 2048;
constexpr int64_t kRecWords = (int64_t)(sizeof(SmqSizeRecord) / 8);  // 16
static_assert(sizeof(SmqSizeRecord) == 128, "SmqSizeRecord layout");
struct RecPool {
  int dev = -1;
  hipStream_t st = nullptr;
  at::Tensor buf;  // int64 [kPoolRecs * kRecWords]
  int64_t next = kPoolRecs;
};
RecPool g_rec_pool;

// A counted call's log_size values as the logger gets them: 0-dim fp64 device views of its record.
struct RecValues {
  at::Tensor ratio, new_size, orig_size;
};

// A 0-dim view of element off of buf, built directly (no dispatcher round trip: select() cost
// ~0.5 us of host time per view, three per counted call). A plain tensor sharing buf's storage,
// as select() returns for a buf that does not require grad.
at::Tensor scalar_view(const at::Tensor& buf, int64_t off) {
  auto impl = c10::make_intrusive<c10::TensorImpl>(c10::Storage(buf.storage()), buf.key_set(),
                                                   buf.dtype());
  impl->set_storage_offset(off);
  impl->set_sizes_contiguous({});
  return at::Tensor(std::move(impl));
}

// The next record (its device pointer) and the views of its values.
SmqSizeRecord* rec_take(const at::Tensor& like, hipStream_t st, RecValues* values) {
  RecPool& P = g_rec_pool;
  const int dev = like.get_device();
  if (P.next >= kPoolRecs || P.dev != dev || P.st != st) {
    P.buf = at::zeros({kPoolRecs * kRecWords}, like.options().dtype(at::kDouble));
    P.dev = dev;
    P.st = st;
    P.next = 0;
  }
  const int64_t i = P.next++;
  const int64_t v = i * kRecWords + (int64_t)(offsetof(SmqSizeRecord, n_outlier) / 8);
  values->new_size = scalar_view(P.buf, v + 1);
  values->ratio = scalar_view(P.buf, v + 2);
  values->orig_size = scalar_view(P.buf, v + 3);
  return reinterpret_cast<SmqSizeRecord*>(P.buf.data_ptr<double>() + i * kRecWords);
}

// rng.__dict__ holds seed / offset (smart_compress_amd/_native.py RngState); the call takes n
// positions of the stream, under the GIL, as RngState.take.
PyObject* g_seed = nullptr;
PyObject* g_offset = nullptr;
PyObject* g_tag = nullptr;
PyObject* g_bwd_tag = nullptr;

bool rng_take(PyObject* rng_dict, uint64_t n, uint64_t* seed, uint64_t* offset) {
  PyObject* s = PyDict_GetItem(rng_dict, g_seed);
  PyObject* o = PyDict_GetItem(rng_dict, g_offset);
  if (!s || !o) {
    PyErr_SetString(PyExc_AttributeError, "RngState without seed / offset");
    return false;
  }
  *seed = PyLong_AsUnsignedLongLongMask(s);
  *offset = PyLong_AsUnsignedLongLongMask(o);
  if (PyErr_Occurred()) return false;
  PyObject* nv = PyLong_FromUnsignedLongLong(*offset + n);  // mod 2^64, as RngState.take
  if (!nv) return false;
  const int rc = PyDict_SetItem(rng_dict, g_offset, nv);
  Py_DECREF(nv);
  return rc == 0;
}

// ---- SmartFP ----------------------------------------------------------------------------------
constexpr int kSnap = 11;
const char* const kSnapKeys[kSnap] = {
    "num_bits_main", "num_bits_outlier", "main_std_dev_threshold", "outlier_std_dev_threshold",
    "stochastic_rounding", "use_range_std_dev", "measure_compression_ratio", "use_sample_stats",
    "min_size", "precision", "use_batch_norm"};
PyObject* g_snap_keys[kSnap];

struct SmaqState {
  SmqSmaqParams tmpl[2];  // [all_positive]
  int64_t min_size = 8;
  bool allow_f16 = false;  // precision 16 (smart.py:154's clamp on a half tensor otherwise raises)
  bool use_bn = false;
  bool decline = false;    // range or sampled statistics: the Python path
  bool count = false;      // --measure_compression_ratio: counted calls (smq_smaq_roundtrip_counted)
  PyRef hp_dict;           // hparams.__dict__
  PyRef snap[kSnap];       // its values when the templates were built
  PyRef rng_dict;          // codec.rng.__dict__
  PyRef ws_getter;
  WsSlot ws;
  WsSlot pws;  // the packed codec's workspace (smaq_packed)
};
using StatePtr = std::shared_ptr<SmaqState>;

void state_capsule_free(PyObject* cap) {
  delete static_cast<StatePtr*>(PyCapsule_GetPointer(cap, "smq.SmaqState"));
}

StatePtr* state_of(PyObject* cap) {
  return static_cast<StatePtr*>(PyCapsule_GetPointer(cap, "smq.SmaqState"));
}

// smaq_state(template_bytes_allpos0, template_bytes_allpos1, hparams_dict, rng_dict, ws_getter
//            [, allow_count]): allow_count False — the ratio-logging calls decline (a subclass
//            codec whose log_size values are not SmartFP's)
PyObject* smaq_state(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 5 && nargs != 6) {
    PyErr_SetString(PyExc_TypeError,
                    "smaq_state(tmpl0, tmpl1, hparams_dict, rng_dict, ws_getter[, allow_count])");
    return nullptr;
  }
  const int allow_count = nargs == 6 ? PyObject_IsTrue(a[5]) : 1;
  if (allow_count < 0) return nullptr;
  Py_buffer b0, b1;
  if (PyObject_GetBuffer(a[0], &b0, PyBUF_SIMPLE) < 0) return nullptr;
  if (PyObject_GetBuffer(a[1], &b1, PyBUF_SIMPLE) < 0) {
    PyBuffer_Release(&b0);
    return nullptr;
  }
  const bool ok = b0.len == (Py_ssize_t)sizeof(SmqSmaqParams) &&
                  b1.len == (Py_ssize_t)sizeof(SmqSmaqParams) && PyDict_Check(a[2]) &&
                  PyDict_Check(a[3]) && PyCallable_Check(a[4]);
  if (!ok) {
    PyBuffer_Release(&b0);
    PyBuffer_Release(&b1);
    PyErr_SetString(PyExc_TypeError, "smaq_state: bad arguments");
    return nullptr;
  }
  auto s = std::make_shared<SmaqState>();
  memcpy(&s->tmpl[0], b0.buf, sizeof(SmqSmaqParams));
  memcpy(&s->tmpl[1], b1.buf, sizeof(SmqSmaqParams));
  PyBuffer_Release(&b0);
  PyBuffer_Release(&b1);
  s->hp_dict.o = a[2];
  Py_INCREF(a[2]);
  for (int i = 0; i < kSnap; ++i) {
    PyObject* v = PyDict_GetItem(a[2], g_snap_keys[i]);  // borrowed (or NULL: absent)
    Py_XINCREF(v);
    s->snap[i].o = v;
  }
  // min_size / precision other than Python ints (a hand-built Namespace, a config file): the
  // Python path, which accepts them, serves the calls
  if (s->snap[8].o) {
    s->min_size = PyLong_Check(s->snap[8].o) ? PyLong_AsLongLong(s->snap[8].o) : -1;
    if (s->min_size == -1 && (PyErr_Occurred() || !PyLong_Check(s->snap[8].o))) {
      PyErr_Clear();
      s->decline = true;
    }
  }
  if (s->snap[9].o) {
    const long prec = PyLong_Check(s->snap[9].o) ? PyLong_AsLong(s->snap[9].o) : -1;
    if (prec == -1 && (PyErr_Occurred() || !PyLong_Check(s->snap[9].o))) {
      PyErr_Clear();
      s->decline = true;
    }
    s->allow_f16 = prec == 16;
  }
  s->use_bn = s->snap[10].o && PyObject_IsTrue(s->snap[10].o) == 1;
  for (int i = 5; i <= 7; i += 2)  // use_range_std_dev, use_sample_stats
    if (s->snap[i].o && PyObject_IsTrue(s->snap[i].o) == 1) s->decline = true;
  s->count = s->snap[6].o && PyObject_IsTrue(s->snap[6].o) == 1;  // measure_compression_ratio
  if (s->count && !allow_count) s->decline = true;
  s->rng_dict.o = a[3];
  Py_INCREF(a[3]);
  s->ws_getter.o = a[4];
  Py_INCREF(a[4]);
  if (PyErr_Occurred()) return nullptr;
  auto* holder = new StatePtr(std::move(s));
  PyObject* cap = PyCapsule_New(holder, "smq.SmaqState", state_capsule_free);
  if (!cap) delete holder;
  return cap;
}

enum RunResult { kError = -1, kDecline = 0, kDone = 1, kStale = 2 };

// One SmartFP call on t (GIL held): kDone with *out set, kDecline (the Python path handles it),
// kStale (the hparams changed since the state was built), kError (Python error set).
// rec: with ratio logging, the call's compression_ratio / new_size / orig_size (0-dim fp64 device
// views of its record); a caller that passes none gets kDecline for a counting codec.
RunResult smaq_run(SmaqState& s, const at::Tensor& t, bool all_positive, at::Tensor* out,
                   RecValues* rec = nullptr) {
  for (int i = 0; i < kSnap; ++i)
    if (PyDict_GetItem(s.hp_dict.o, g_snap_keys[i]) != s.snap[i].o) return kStale;
  if (s.decline || !t.is_cuda() || (s.count && !rec)) return kDecline;
  int code;
  switch (t.scalar_type()) {
    case at::kFloat: code = SMQ_DTYPE_F32; break;
    case at::kBFloat16: code = SMQ_DTYPE_BF16; break;
    case at::kHalf:
      if (!s.allow_f16) return kDecline;
      code = SMQ_DTYPE_F16;
      break;
    default: return kDecline;
  }
  const int64_t n = t.numel();
  if (n < s.min_size) return kDecline;
  at::Tensor x = t.is_contiguous() ? t : t.detach().contiguous();
  const int dev = x.get_device();
  const hipStream_t st = c10::hip::getCurrentHIPStream(dev).stream();
  if (!ws_lookup(s.ws, s.ws_getter.o, dev, st, smq_smaq_workspace_bytes(n))) return kError;
  SmqSmaqParams p = s.tmpl[all_positive ? 1 : 0];
  if (!rng_take(s.rng_dict.o, (uint64_t)n, &p.seed, &p.offset)) return kError;
  if (s.count) {  // a graph capture would keep the pool's records: the Python path refuses it
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
      return kDecline;
  }
  at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  int rc;
  if (s.count) {
    SmqSizeRecord* r = rec_take(x, st, rec);
    rc = smq_smaq_roundtrip_counted(x.const_data_ptr(), code, y.mutable_data_ptr<float>(), n, &p,
                                    s.ws.ptr, s.ws.bytes, r, st);
  } else {
    rc = smq_smaq_roundtrip(x.const_data_ptr(), code, y.mutable_data_ptr<float>(), n, &p, nullptr,
                            s.ws.ptr, s.ws.bytes, st);
  }
  if (rc) {
    PyErr_Format(PyExc_RuntimeError, "smq_smaq_roundtrip failed (rc=%d): %s", rc,
                 smq_last_error());
    return kError;
  }
  *out = std::move(y);
  return kDone;
}

PyObject* g_log_rec = nullptr;  // "_log_size_record"
PyObject* g_fwd_tag = nullptr;  // "forward_autograd"

// (ratio, new_size, orig_size) as a new tuple of tensors, or NULL (Python error set)
PyObject* rec_tuple(RecValues&& v) {
  PyObject* a = THPVariable_Wrap(std::move(v.ratio));
  PyObject* b = a ? THPVariable_Wrap(std::move(v.new_size)) : nullptr;
  PyObject* c = b ? THPVariable_Wrap(std::move(v.orig_size)) : nullptr;
  PyObject* r = c ? PyTuple_Pack(3, a, b, c) : nullptr;
  Py_XDECREF(a);
  Py_XDECREF(b);
  Py_XDECREF(c);
  return r;
}

// codec._log_size_record(tag, ratio, new_size, orig_size) (GIL held): the counted call's log_size,
// values on the device
bool log_record(PyObject* codec, PyObject* tag, RecValues&& rec) {
  PyObject* a = THPVariable_Wrap(std::move(rec.ratio));
  PyObject* b = a ? THPVariable_Wrap(std::move(rec.new_size)) : nullptr;
  PyObject* c = b ? THPVariable_Wrap(std::move(rec.orig_size)) : nullptr;
  PyObject* r = c ? PyObject_CallMethodObjArgs(codec, g_log_rec, tag, a, b, c, nullptr) : nullptr;
  Py_XDECREF(a);
  Py_XDECREF(b);
  Py_XDECREF(c);
  Py_XDECREF(r);
  return r != nullptr;
}

// smaq(state, x, all_positive, batch_norm_stats) -> y | None (not handled here) |
// NotImplemented (the hparams changed: rebuild the state)
PyObject* smaq(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "smaq(state, x, all_positive, batch_norm_stats)");
    return nullptr;
  }
  StatePtr* sp = state_of(a[0]);
  if (!sp) return nullptr;
  SmaqState& s = **sp;
  if (a[3] != Py_None && s.use_bn) Py_RETURN_NONE;
  if (!THPVariable_Check(a[1])) Py_RETURN_NONE;
  const int ap = PyObject_IsTrue(a[2]);
  if (ap < 0) return nullptr;
  at::Tensor y;
  RecValues rec;
  switch (smaq_run(s, THPVariable_Unpack(a[1]), ap != 0, &y, &rec)) {
    case kDone: break;
    case kDecline: Py_RETURN_NONE;
    case kStale: Py_RETURN_NOTIMPLEMENTED;
    default: return nullptr;
  }
  if (!s.count) return THPVariable_Wrap(std::move(y));
  // ratio logging: (y, (ratio, new_size, orig_size)) — the codec logs them under the call's tag
  PyObject* yo = THPVariable_Wrap(std::move(y));
  PyObject* ro = yo ? rec_tuple(std::move(rec)) : nullptr;
  if (!ro) {
    Py_XDECREF(yo);
    return nullptr;
  }
  PyObject* r = PyTuple_Pack(2, yo, ro);
  Py_DECREF(yo);
  Py_DECREF(ro);
  return r;
}

// Bytes of a stream of n elements with every element an outlier and escape_frac of them escaped
// (util/pytorch/saved.py stream_capacity, the same integer arithmetic).
size_t stream_capacity(int64_t n, int bm, int bo, double escape_frac) {
  const int64_t nb = (n + SMQ_PACK_BLOCK - 1) / SMQ_PACK_BLOCK;
  const int64_t wm = bm - 1, wo = bo - 1, we = wo > wm ? wo - wm : 0;
  const int64_t fixed_words = 128 + 128 * wm;
  const int64_t var_words = (we * n + 31) / 32 + nb + 2 * ((int64_t)(escape_frac * (double)n) + nb);
  return (size_t)((int64_t)sizeof(SmqPackedHeader) + 8 * (nb + (nb & 1)) +
                  4 * (nb * fixed_words + var_words));
}

// PackedActivations' forward call on t (GIL held): y as smaq_run computes it and its stream
// (smq_smaq_roundtrip_compress_notify) in a new buffer of stream_capacity bytes, its size also into
// *notify (NULL: not). The same declines as smaq_run (and ratio logging: PackedActivations logs the
// stream's own size).
RunResult packed_run(SmaqState& s, const at::Tensor& t, bool ap, PyObject* getter, double frac,
                     uint32_t* notify, at::Tensor* y_out, at::Tensor* data_out) {
  for (int i = 0; i < kSnap; ++i)
    if (PyDict_GetItem(s.hp_dict.o, g_snap_keys[i]) != s.snap[i].o) return kStale;
  if (s.decline || s.count || !t.is_cuda()) return kDecline;
  int code;
  switch (t.scalar_type()) {
    case at::kFloat: code = SMQ_DTYPE_F32; break;
    case at::kBFloat16: code = SMQ_DTYPE_BF16; break;
    case at::kHalf:
      if (!s.allow_f16) return kDecline;
      code = SMQ_DTYPE_F16;
      break;
    default: return kDecline;
  }
  const int64_t n = t.numel();
  if (n < s.min_size) return kDecline;
  at::Tensor x = t.is_contiguous() ? t : t.detach().contiguous();
  const int dev = x.get_device();
  const hipStream_t st = c10::hip::getCurrentHIPStream(dev).stream();
  if (!ws_lookup(s.pws, getter, dev, st, smq_smaq_pack_workspace_bytes(n))) return kError;
  SmqSmaqParams p = s.tmpl[ap ? 1 : 0];
  const size_t cap = stream_capacity(n, p.num_bits_main, p.num_bits_outlier, frac);
  if (!rng_take(s.rng_dict.o, (uint64_t)n, &p.seed, &p.offset)) return kError;
  at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  at::Tensor data = at::empty({(int64_t)cap}, x.options().dtype(at::kByte));
  const int rc = smq_smaq_roundtrip_compress_notify(
      x.const_data_ptr(), code, y.mutable_data_ptr<float>(), n, &p, data.mutable_data_ptr(), cap,
      s.pws.ptr, s.pws.bytes, notify, st);
  if (rc) {
    PyErr_Format(PyExc_RuntimeError, "smq_smaq_roundtrip_compress_notify failed (rc=%d): %s", rc,
                 smq_last_error());
    return kError;
  }
  *y_out = std::move(y);
  *data_out = std::move(data);
  return kDone;
}

// (y, data) as a new tuple, or NULL
PyObject* pair_of(at::Tensor&& y, at::Tensor&& data) {
  PyObject* yo = THPVariable_Wrap(std::move(y));
  PyObject* dobj = yo ? THPVariable_Wrap(std::move(data)) : nullptr;
  if (!dobj) {
    Py_XDECREF(yo);
    return nullptr;
  }
  PyObject* r = PyTuple_Pack(2, yo, dobj);
  Py_DECREF(yo);
  Py_DECREF(dobj);
  return r;
}

// The optional notify argument: None or the address (an int) of a host-mapped word; false on a
// Python error.
bool notify_arg(PyObject* const* a, Py_ssize_t nargs, Py_ssize_t i, uint32_t** out) {
  *out = nullptr;
  if (nargs <= i || a[i] == Py_None) return true;
  *out = (uint32_t*)PyLong_AsVoidPtr(a[i]);
  return !PyErr_Occurred();
}

// smaq_packed(state, x, all_positive, pack_ws_getter, escape_frac[, notify]) -> (y, stream) | None
// | NotImplemented: PackedActivations' forward call (util/pytorch/saved.py) in one C call.
PyObject* smaq_packed(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 5 && nargs != 6) {
    PyErr_SetString(PyExc_TypeError,
                    "smaq_packed(state, x, all_positive, getter, escape_frac[, notify])");
    return nullptr;
  }
  uint32_t* notify;
  if (!notify_arg(a, nargs, 5, &notify)) return nullptr;
  StatePtr* sp = state_of(a[0]);
  if (!sp) return nullptr;
  if (!THPVariable_Check(a[1])) Py_RETURN_NONE;
  const int ap = PyObject_IsTrue(a[2]);
  if (ap < 0) return nullptr;
  const double frac = PyFloat_AsDouble(a[4]);
  if (frac == -1.0 && PyErr_Occurred()) return nullptr;
  at::Tensor y, data;
  switch (packed_run(**sp, THPVariable_Unpack(a[1]), ap != 0, a[3], frac, notify, &y, &data)) {
    case kDone: return pair_of(std::move(y), std::move(data));
    case kDecline: Py_RETURN_NONE;
    case kStale: Py_RETURN_NOTIMPLEMENTED;
    default: return nullptr;
  }
}

// smaq_unpacked(data, shape, n, num_bits_main, num_bits_outlier) -> y: PackedActivations' backward
// decode (SmartFPPacked.decompress of a device stream written with these widths) in one C call: y
// allocated with the stream's shape, smq_smaq_decompress_ex on the current stream.
PyObject* smaq_unpacked(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 5 || !THPVariable_Check(a[0]) || !PyTuple_Check(a[1])) {
    PyErr_SetString(PyExc_TypeError, "smaq_unpacked(data, shape, n, bm, bo)");
    return nullptr;
  }
  const at::Tensor& data = THPVariable_Unpack(a[0]);
  if (!data.is_cuda()) {
    PyErr_SetString(PyExc_ValueError, "smaq_unpacked: the stream must be on a ROCm device");
    return nullptr;
  }
  const Py_ssize_t nd = PyTuple_GET_SIZE(a[1]);
  std::vector<int64_t> shape((size_t)nd);
  for (Py_ssize_t i = 0; i < nd; ++i) shape[(size_t)i] = PyLong_AsLongLong(PyTuple_GET_ITEM(a[1], i));
  const int64_t n = PyLong_AsLongLong(a[2]);
  const int bm = (int)PyLong_AsLong(a[3]), bo = (int)PyLong_AsLong(a[4]);
  if (PyErr_Occurred()) return nullptr;
  const int dev = data.get_device();
  const hipStream_t st = c10::hip::getCurrentHIPStream(dev).stream();
  at::Tensor y = at::empty(shape, data.options().dtype(at::kFloat));
  const int rc = smq_smaq_decompress_ex(data.const_data_ptr(), y.mutable_data_ptr<float>(), n, bm,
                                        bo, st);
  if (rc) {
    PyErr_Format(PyExc_RuntimeError, "smq_smaq_decompress_ex failed (rc=%d): %s", rc,
                 smq_last_error());
    return nullptr;
  }
  return THPVariable_Wrap(std::move(y));
}

// ---- the autograd wrapper (autograd.py:18-47: Compressor with a SmartFP compress_fn) -----------
// The backward of `y = compress(x)` is `compress(grad_y)` (tag "backward_autograd"); with the
// backward direction switched off the grad passes unchanged (autograd.py:40-41).
struct SmaqCompressBackward : public torch::autograd::Node {
  StatePtr state;   // nullptr: backward compression off
  PyRef codec;      // the Python codec: what the C path declines or a stale state goes to

  torch::autograd::variable_list apply(torch::autograd::variable_list&& grads) override {
    at::Tensor g = grads[0];
    if (!task_should_compute_output(0)) return {at::Tensor()};
    if (!g.defined() || !state) return {g};
    PyGILState_STATE gs = PyGILState_Ensure();
    at::Tensor out;
    RecValues rec;
    RunResult r = smaq_run(*state, g, false, &out, &rec);
    if (r == kDone && state->count && !log_record(codec.o, g_bwd_tag, std::move(rec))) r = kError;
    if (r == kDecline || r == kStale) {  // the codec's own call (it rebuilds a stale state)
      PyObject* gv = THPVariable_Wrap(g);
      PyObject* res = nullptr;
      if (gv) {
        PyObject* args = PyTuple_Pack(1, gv);
        PyObject* kw = args ? PyDict_New() : nullptr;
        if (kw && PyDict_SetItem(kw, g_tag, g_bwd_tag) == 0)
          res = PyObject_Call(codec.o, args, kw);
        Py_XDECREF(kw);
        Py_XDECREF(args);
        Py_DECREF(gv);
      }
      if (res && THPVariable_Check(res)) {
        out = THPVariable_Unpack(res);
        r = kDone;
      } else {
        if (res) PyErr_SetString(PyExc_TypeError, "codec returned a non-tensor");
        r = kError;
      }
      Py_XDECREF(res);
    }
    if (r != kDone) {
      std::string msg = "SmaqCompressBackward: codec call failed";
      PyObject *t, *v, *tb;
      PyErr_Fetch(&t, &v, &tb);
      if (v) {
        PyObject* str = PyObject_Str(v);
        if (str) {
          const char* c = PyUnicode_AsUTF8(str);
          if (c) msg += std::string(": ") + c;
          Py_DECREF(str);
        }
      }
      Py_XDECREF(t);
      Py_XDECREF(v);
      Py_XDECREF(tb);
      PyErr_Clear();
      PyGILState_Release(gs);
      throw std::runtime_error(msg);
    }
    PyGILState_Release(gs);
    return {out};
  }
  std::string name() const override { return "SmaqCompressBackward"; }
};

// smaq_autograd(state, x, codec, backward) -> y | None | NotImplemented: Compressor.forward for
// x alone (no batch_norm_stats argument); y carries a SmaqCompressBackward node when x requires
// grad and grad mode is on.
PyObject* smaq_autograd(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "smaq_autograd(state, x, codec, backward)");
    return nullptr;
  }
  StatePtr* sp = state_of(a[0]);
  if (!sp) return nullptr;
  if (!THPVariable_Check(a[1])) Py_RETURN_NONE;
  const int bwd = PyObject_IsTrue(a[3]);
  if (bwd < 0) return nullptr;
  const at::Tensor& x = THPVariable_Unpack(a[1]);
  at::Tensor y;
  RecValues rec;
  switch (smaq_run(**sp, x, false, &y, &rec)) {
    case kDone: break;
    case kDecline: Py_RETURN_NONE;
    case kStale: Py_RETURN_NOTIMPLEMENTED;
    default: return nullptr;
  }
  if ((*sp)->count && !log_record(a[2], g_fwd_tag, std::move(rec))) return nullptr;
  if (torch::autograd::compute_requires_grad(x)) {
    auto node = std::shared_ptr<SmaqCompressBackward>(new SmaqCompressBackward(),
                                                      torch::autograd::deleteNode);
    if (bwd) node->state = *sp;
    node->codec.o = a[2];
    Py_INCREF(a[2]);
    node->set_next_edges(torch::autograd::collect_next_edges(x));
    torch::autograd::set_history(y, node);
  }
  return THPVariable_Wrap(std::move(y));
}

// smaq_packed_autograd(state, x, acts, backward, pack_ws_getter, escape_frac[, notify]) ->
// (y, stream) | None | NotImplemented: Compressor.forward with PackedActivations inside its context
// (util/pytorch/saved.py): the packed forward call (packed_run) and the SmaqCompressBackward node,
// whose backward is the codec's plain call on the grad-map (what PackedActivations does for
// backward-direction calls); its declines go to acts(grad, tag="backward_autograd").
PyObject* smaq_packed_autograd(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 6 && nargs != 7) {
    PyErr_SetString(PyExc_TypeError,
                    "smaq_packed_autograd(state, x, acts, backward, getter, escape_frac[, notify])");
    return nullptr;
  }
  uint32_t* notify;
  if (!notify_arg(a, nargs, 6, &notify)) return nullptr;
  StatePtr* sp = state_of(a[0]);
  if (!sp) return nullptr;
  if (!THPVariable_Check(a[1])) Py_RETURN_NONE;
  const int bwd = PyObject_IsTrue(a[3]);
  if (bwd < 0) return nullptr;
  const double frac = PyFloat_AsDouble(a[5]);
  if (frac == -1.0 && PyErr_Occurred()) return nullptr;
  const at::Tensor& x = THPVariable_Unpack(a[1]);
  at::Tensor y, data;
  switch (packed_run(**sp, x, false, a[4], frac, notify, &y, &data)) {
    case kDone: break;
    case kDecline: Py_RETURN_NONE;
    case kStale: Py_RETURN_NOTIMPLEMENTED;
    default: return nullptr;
  }
  if (torch::autograd::compute_requires_grad(x)) {
    auto node = std::shared_ptr<SmaqCompressBackward>(new SmaqCompressBackward(),
                                                      torch::autograd::deleteNode);
    if (bwd) node->state = *sp;
    node->codec.o = a[2];
    Py_INCREF(a[2]);
    node->set_next_edges(torch::autograd::collect_next_edges(x));
    torch::autograd::set_history(y, node);
  }
  return pair_of(std::move(y), std::move(data));
}

// ---- S2FP8 (fp32 device tensors at precision 32, s2fp8.py:27-48) --------------------------------
WsSlot g_s2_ws;

// s2fp8(x, check_inf, rng_dict, ws_getter) -> y | None (not an fp32 device tensor)
PyObject* s2fp8(PyObject*, PyObject* const* a, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "s2fp8(x, check_inf, rng_dict, ws_getter)");
    return nullptr;
  }
  if (!THPVariable_Check(a[0]) || !PyDict_Check(a[2])) Py_RETURN_NONE;
  const at::Tensor& t = THPVariable_Unpack(a[0]);
  if (!t.is_cuda() || t.scalar_type() != at::kFloat) Py_RETURN_NONE;
  const int64_t n = t.numel();
  const int check_inf = PyObject_IsTrue(a[1]);
  if (check_inf < 0) return nullptr;
  at::Tensor x = t.is_contiguous() ? t : t.detach().contiguous();
  at::Tensor y = at::empty(x.sizes(), x.options());
  if (n == 0) return THPVariable_Wrap(std::move(y));
  const int dev = x.get_device();
  const hipStream_t st = c10::hip::getCurrentHIPStream(dev).stream();
  if (!ws_lookup(g_s2_ws, a[3], dev, st, smq_s2fp8_workspace_bytes(1))) return nullptr;
  uint64_t seed, offset;
  if (!rng_take(a[2], (uint64_t)n, &seed, &offset)) return nullptr;
  const int rc = smq_s2fp8_roundtrip(x.const_data_ptr(), SMQ_DTYPE_F32, y.mutable_data_ptr(), n, 32,
                                     check_inf, nullptr, seed, offset, nullptr, nullptr,
                                     g_s2_ws.ptr, g_s2_ws.bytes, st);
  if (rc) {
    PyErr_Format(PyExc_RuntimeError, "smq_s2fp8_roundtrip failed (rc=%d): %s", rc,
                 smq_last_error());
    return nullptr;
  }
  return THPVariable_Wrap(std::move(y));
}

PyMethodDef kMethods[] = {
    {"smaq_state", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq_state)),
     METH_FASTCALL, "SmartFP hot-path state from its parameter templates and hparams"},
    {"smaq", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq)), METH_FASTCALL,
     "one eager SmartFP call (smq_smaq_roundtrip), or None / NotImplemented"},
    {"smaq_autograd",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq_autograd)), METH_FASTCALL,
     "Compressor.forward with a SmartFP codec: y and its SmaqCompressBackward node"},
    {"smaq_packed", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq_packed)),
     METH_FASTCALL, "PackedActivations' forward call: (y, stream) (smq_smaq_roundtrip_compress)"},
    {"smaq_packed_autograd",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq_packed_autograd)),
     METH_FASTCALL, "Compressor.forward with PackedActivations: (y, stream), y with its node"},
    {"smaq_unpacked",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(smaq_unpacked)), METH_FASTCALL,
     "PackedActivations' backward decode of a device stream (smq_smaq_decompress_ex)"},
    {"s2fp8", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(s2fp8)), METH_FASTCALL,
     "one eager S2FP8 call on an fp32 device tensor (smq_s2fp8_roundtrip), or None"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_smqtorch", nullptr, -1, kMethods,
                       nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__smqtorch(void) {
  g_seed = PyUnicode_InternFromString("seed");
  g_offset = PyUnicode_InternFromString("offset");
  g_tag = PyUnicode_InternFromString("tag");
  g_bwd_tag = PyUnicode_InternFromString("backward_autograd");
  g_fwd_tag = PyUnicode_InternFromString("forward_autograd");
  g_log_rec = PyUnicode_InternFromString("_log_size_record");
  for (int i = 0; i < kSnap; ++i) g_snap_keys[i] = PyUnicode_InternFromString(kSnapKeys[i]);
  return PyModule_Create(&kModule);
}
