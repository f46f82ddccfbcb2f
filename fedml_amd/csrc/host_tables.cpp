// host_tables.cpp -- host-side helper of the aggregation engine's Python binding (CPU code only).
//
// A state_dict round hands the engine K client dicts x T keys = K*T tensors (ViT-B/16 at K=128:
// 19,456).  Walking them in Python to validate and collect data pointers costs ~1 us per tensor,
// i.e. longer than the GPU takes to aggregate them.  This helper does the walk in C++ (tens of ns
// per tensor) and also carves the outputs out of one device allocation.  It touches tensor DATA in
// one place only: small_host_round's host-resident rounds below the measured break-even size
// (host_sum.h: the kernels' per-element contract on the CPU that already holds the data, where a
// PCIe round trip alone costs more than the reference's whole CPU loop); every other round's
// arithmetic is in the HIP kernels behind the C ABI (include/fedagg.h).
#include <torch/extension.h>

#include "host_sum.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

int fa_dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    case at::kDouble: return 3;
    case at::kLong: return 4;
    default: return -1;
  }
}

}  // namespace

// gather(dicts, keys) -> (ptrs int64[T*K] key-major, numel int64[T], codes int64[T], shapes, device)
//  * KeyError if a client lacks a key (as the reference's `local_model_params[k]`);
//  * TypeError if clients disagree on a key's dtype, RuntimeError on a shape mismatch;
//  * every tensor must be contiguous and on the device of client 0's first tensor;
//  * code -1 marks dtypes the C ABI does not take natively (the caller widens those).
py::tuple gather(py::list dicts, py::list keys) {
  const int64_t K = (int64_t)py::len(dicts);
  const int64_t T = (int64_t)py::len(keys);
  if (K == 0) throw py::index_error("list index out of range");
  auto ptrs = torch::empty({T * K}, torch::kInt64);
  auto numel = torch::empty({T}, torch::kInt64);
  auto codes = torch::empty({T}, torch::kInt64);
  int64_t* P = ptrs.data_ptr<int64_t>();
  int64_t* Nn = numel.data_ptr<int64_t>();
  int64_t* C = codes.data_ptr<int64_t>();
  std::vector<PyObject*> kv(T);
  for (int64_t t = 0; t < T; ++t) kv[t] = PyList_GET_ITEM(keys.ptr(), t);
  std::vector<at::ScalarType> st(T);
  std::vector<std::vector<int64_t>> shape(T);
  py::list shapes;
  c10::optional<at::Device> dev;
  std::vector<PyObject*> items(T);
  auto key_name = [&](int64_t t) { return py::str(kv[t]).cast<std::string>(); };
  // Client-major walk.  A client's state_dict normally lists client 0's keys in the same order, so
  // its values are read with PyDict_Next and one key comparison each (identity or string equality);
  // any other dict falls back to per-key lookups (the reference's `local_model_params[k]`).
  for (int64_t i = 0; i < K; ++i) {
    PyObject* d = PyList_GET_ITEM(dicts.ptr(), i);
    if (!PyDict_Check(d)) throw py::type_error("state_dicts must be dicts");
    bool in_order = PyDict_GET_SIZE(d) == T;
    if (in_order) {
      Py_ssize_t pos = 0;
      PyObject *k, *v;
      for (int64_t t = 0; t < T && in_order; ++t) {
        if (!PyDict_Next(d, &pos, &k, &v)) { in_order = false; break; }
        if (k != kv[t]) {
          const int eq = PyObject_RichCompareBool(k, kv[t], Py_EQ);
          if (eq < 0) throw py::error_already_set();
          if (!eq) { in_order = false; break; }
        }
        items[t] = v;
      }
    }
    if (!in_order) {
      for (int64_t t = 0; t < T; ++t) {
        PyObject* v = PyDict_GetItemWithError(d, kv[t]);
        if (!v) {
          if (PyErr_Occurred()) throw py::error_already_set();
          throw py::key_error(key_name(t));
        }
        items[t] = v;
      }
    }
    for (int64_t t = 0; t < T; ++t) {
      PyObject* item = items[t];
      if (!THPVariable_Check(item)) throw py::type_error("state_dict values must be tensors");
      const at::Tensor& x = THPVariable_Unpack(item);
      if (i == 0) {
        st[t] = x.scalar_type();
        shape[t] = x.sizes().vec();
        if (!dev) dev = x.device();
        Nn[t] = x.numel();
        C[t] = fa_dtype_code(st[t]);
        shapes.append(py::cast(shape[t]));
      } else {
        if (x.scalar_type() != st[t])
          throw py::type_error("key " + key_name(t) + ": client " + std::to_string(i) +
                               " has a different dtype than client 0");
        if (x.sizes() != c10::IntArrayRef(shape[t]))
          throw std::runtime_error("key " + key_name(t) + ": client " + std::to_string(i) +
                                   " shape differs from client 0");
      }
      if (x.device() != *dev)
        throw std::invalid_argument("key " + key_name(t) + ": client " + std::to_string(i) +
                                    " is on another device than client 0");
      if (!x.is_contiguous())
        throw std::invalid_argument("key " + key_name(t) + ": client " + std::to_string(i) + " is not contiguous");
      P[t * K + i] = (int64_t)x.data_ptr();
    }
  }
  std::string devs = dev ? dev->str() : std::string("cpu");
  return py::make_tuple(ptrs, numel, codes, shapes, devs);
}

// alloc_outputs(shapes, dtypes, device) -> (arena, views, ptrs int64[T])
// One device allocation; every output starts on a 256-byte boundary (vector path of the kernel).
py::tuple alloc_outputs(py::list shapes, py::list dtypes, const std::string& device) {
  const int64_t T = (int64_t)py::len(shapes);
  std::vector<int64_t> off(T), nbytes(T);
  std::vector<at::ScalarType> sts(T);
  std::vector<std::vector<int64_t>> shp(T);
  int64_t total = 0;
  for (int64_t t = 0; t < T; ++t) {
    shp[t] = shapes[t].cast<std::vector<int64_t>>();
    sts[t] = torch::python::detail::py_object_to_dtype(dtypes[t]);
    int64_t n = 1;
    for (auto s : shp[t]) n *= s;
    nbytes[t] = n * (int64_t)c10::elementSize(sts[t]);
    off[t] = total;
    total += (nbytes[t] + 255) / 256 * 256;
  }
  auto arena = torch::empty({std::max<int64_t>(total, 256)}, torch::TensorOptions().dtype(torch::kUInt8).device(device));
  // Views are built directly on the arena's storage (one TensorImpl each, ~10x cheaper than
  // narrow().view(dtype).view(shape), which dominated a 122-key round's host time).
  const c10::Storage& storage = arena.storage();
  const c10::DispatchKeySet keys = arena.key_set();
  char* base = (char*)arena.data_ptr();
  py::list views;
  auto ptrs = torch::empty({T}, torch::kInt64);
  int64_t* P = ptrs.data_ptr<int64_t>();
  for (int64_t t = 0; t < T; ++t) {
    at::Tensor v = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(storage), keys,
                                                            caffe2::TypeMeta::fromScalarType(sts[t]));
    c10::TensorImpl* impl = v.unsafeGetTensorImpl();
    impl->set_storage_offset(off[t] / (int64_t)c10::elementSize(sts[t]));  // offsets are 256-byte aligned
    impl->set_sizes_contiguous(shp[t]);
    P[t] = (int64_t)(base + off[t]);
    views.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(v))));
  }
  return py::make_tuple(arena, views, ptrs);
}

// plan_outputs(shapes, codes, int64_to_f32, device, ptrs, K) -> (arena, views, groups): the outputs
// of a device round (alloc_outputs, output dtype = input dtype except int64 -> float32 when
// int64_to_f32: the weighted modes' PyTorch promotion) and, per input dtype code in ascending
// order, the launch tables (code, numel int64[Tg], in int64[Tg*K] key-major, out int64[Tg]) --
// what the Python dispatcher had built with a per-key loop and index_select (~50 us a 122-key round).
py::tuple plan_outputs(py::list shapes, torch::Tensor codes, bool int64_to_f32, const std::string& device,
                       torch::Tensor ptrs, int64_t K) {
  const int64_t T = (int64_t)py::len(shapes);
  TORCH_CHECK(codes.dtype() == torch::kInt64 && codes.numel() == T && codes.is_contiguous(), "plan_outputs: codes");
  TORCH_CHECK(ptrs.dtype() == torch::kInt64 && ptrs.numel() == T * K && ptrs.is_contiguous(), "plan_outputs: ptrs");
  const int64_t* C = codes.data_ptr<int64_t>();
  const int64_t* P = ptrs.data_ptr<int64_t>();
  static const at::ScalarType kCode[5] = {at::kFloat, at::kBFloat16, at::kHalf, at::kDouble, at::kLong};
  std::vector<int64_t> off(T), numel(T);
  std::vector<at::ScalarType> sts(T);
  std::vector<std::vector<int64_t>> shp(T);
  int64_t total = 0;
  for (int64_t t = 0; t < T; ++t) {
    TORCH_CHECK(C[t] >= 0 && C[t] <= 4, "plan_outputs: dtype code ", C[t]);
    shp[t] = shapes[t].cast<std::vector<int64_t>>();
    sts[t] = (C[t] == 4 && int64_to_f32) ? at::kFloat : kCode[C[t]];
    int64_t n = 1;
    for (auto x : shp[t]) n *= x;
    numel[t] = n;
    off[t] = total;
    total += (n * (int64_t)c10::elementSize(sts[t]) + 255) / 256 * 256;
  }
  auto arena = torch::empty({std::max<int64_t>(total, 256)}, torch::TensorOptions().dtype(torch::kUInt8).device(device));
  const c10::Storage& storage = arena.storage();
  const c10::DispatchKeySet keys = arena.key_set();
  char* base = (char*)arena.data_ptr();
  py::list views;
  for (int64_t t = 0; t < T; ++t) {
    at::Tensor v = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(storage), keys,
                                                            caffe2::TypeMeta::fromScalarType(sts[t]));
    c10::TensorImpl* impl = v.unsafeGetTensorImpl();
    impl->set_storage_offset(off[t] / (int64_t)c10::elementSize(sts[t]));
    impl->set_sizes_contiguous(shp[t]);
    views.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(v))));
  }
  py::list groups;
  for (int64_t c = 0; c <= 4; ++c) {
    int64_t tg = 0;
    for (int64_t t = 0; t < T; ++t) tg += C[t] == c;
    if (!tg) continue;
    auto nm = torch::empty({tg}, torch::kInt64);
    auto in = torch::empty({tg * K}, torch::kInt64);
    auto out = torch::empty({tg}, torch::kInt64);
    int64_t *N = nm.data_ptr<int64_t>(), *I = in.data_ptr<int64_t>(), *O = out.data_ptr<int64_t>();
    int64_t j = 0;
    for (int64_t t = 0; t < T; ++t) {
      if (C[t] != c) continue;
      N[j] = numel[t];
      std::memcpy(I + j * K, P + t * K, sizeof(int64_t) * (size_t)K);
      O[j] = (int64_t)(base + off[t]);
      ++j;
    }
    groups.append(py::make_tuple(c, nm, in, out));
  }
  return py::make_tuple(arena, views, groups);
}

// carve(flat, offsets, shapes) -> [views]: contiguous views of a flat 1-D tensor at the given
// element offsets (the per-key outputs of an arena's dtype group), built directly on its storage
// like alloc_outputs' (Python slicing + view costs ~3 us a key: a 122-key round's whole kernel time).
py::list carve(torch::Tensor flat, py::list offsets, py::list shapes) {
  TORCH_CHECK(flat.dim() == 1 && flat.is_contiguous(), "carve: flat contiguous 1-D tensor expected");
  const int64_t T = (int64_t)py::len(shapes);
  TORCH_CHECK((int64_t)py::len(offsets) == T, "carve: offsets and shapes differ in length");
  const c10::Storage& storage = flat.storage();
  const c10::DispatchKeySet keys = flat.key_set();
  const caffe2::TypeMeta meta = flat.dtype();
  const int64_t base = flat.storage_offset(), total = flat.numel();
  py::list views;
  for (int64_t t = 0; t < T; ++t) {
    const int64_t off = offsets[t].cast<int64_t>();
    std::vector<int64_t> shp = shapes[t].cast<std::vector<int64_t>>();
    int64_t n = 1;
    for (auto s : shp) n *= s;
    TORCH_CHECK(off >= 0 && n >= 0 && off + n <= total, "carve: view ", t, " out of range");
    at::Tensor v = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(storage), keys, meta);
    c10::TensorImpl* impl = v.unsafeGetTensorImpl();
    impl->set_storage_offset(base + off);
    impl->set_sizes_contiguous(shp);
    views.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(v))));
  }
  return views;
}

// pack_range(src, dst_off, nbytes, lo, hi, dst, nthreads): host-ingest packing.  Job j copies
// nbytes[j] bytes from address src[j] to byte dst_off[j] of a virtual [K, row] staging matrix;
// this call materialises the bytes [lo, hi) of that matrix at address `dst` (dst_off sorted,
// ranges disjoint; bytes no job covers are left untouched).  The copy runs on `nthreads` threads
// with the GIL released: unpickled client tensors sit in pageable memory, and one thread's memcpy
// into pinned staging (~10 GB/s) would otherwise be slower than the PCIe link it feeds.
void pack_range(torch::Tensor src, torch::Tensor dst_off, torch::Tensor nbytes, int64_t lo, int64_t hi,
                int64_t dst, int64_t nthreads) {
  TORCH_CHECK(src.dtype() == torch::kInt64 && dst_off.dtype() == torch::kInt64 && nbytes.dtype() == torch::kInt64,
              "pack_range: int64 job tables");
  TORCH_CHECK(src.is_contiguous() && dst_off.is_contiguous() && nbytes.is_contiguous(), "pack_range: contiguous");
  const int64_t J = src.numel();
  TORCH_CHECK(dst_off.numel() == J && nbytes.numel() == J, "pack_range: table sizes differ");
  const int64_t* S = src.data_ptr<int64_t>();
  const int64_t* D = dst_off.data_ptr<int64_t>();
  const int64_t* B = nbytes.data_ptr<int64_t>();
  char* out = reinterpret_cast<char*>(dst);
  if (hi <= lo || J == 0) return;
  auto work = [&](int64_t a, int64_t b) {  // bytes [a, b) of the matrix
    int64_t j = std::upper_bound(D, D + J, a) - D - 1;  // last job starting at or before a
    if (j < 0) j = 0;
    for (; j < J && D[j] < b; ++j) {
      const int64_t s0 = std::max(a, D[j]), s1 = std::min(b, D[j] + B[j]);
      if (s1 > s0) std::memcpy(out + (s0 - lo), reinterpret_cast<const char*>(S[j]) + (s0 - D[j]), (size_t)(s1 - s0));
    }
  };
  const int64_t total = hi - lo;
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>(nthreads, total / (1 << 20) + 1));
  py::gil_scoped_release nogil;
  if (nt == 1) { work(lo, hi); return; }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t a = lo + total * t / nt, b = lo + total * (t + 1) / nt;
    th.emplace_back(work, a, b);
  }
  for (auto& x : th) x.join();
}

// match_rows(dicts, keys, base, stride, rows) -> bool: does every dict list exactly `keys` (in
// order) with values that are the views of an arena's rows -- value t of dict i at address
// base[t] + rows[i] * stride[t], contiguous?  The arena-resident fast path of a state_dict
// aggregation (fedml_amd/arena.py resident_rows) needs only this, not gather()'s full validation
// and tables: one pass, no allocation, early exit (~10 ns per tensor).
//
// meta: per key t, at meta[moff[t]]: the layout's scalar type, ndim, then the sizes -- a value that
// sits at the right address but was re-viewed with another dtype or shape (x.view(torch.int32),
// x.view(s2)) is not the arena's view, and the pointer-table path handles it.
bool match_rows(py::list dicts, py::list keys, torch::Tensor base, torch::Tensor stride, py::list rows,
                torch::Tensor meta, torch::Tensor moff) {
  const int64_t K = (int64_t)py::len(dicts);
  const int64_t T = (int64_t)py::len(keys);
  TORCH_CHECK(base.dtype() == torch::kInt64 && stride.dtype() == torch::kInt64 && base.numel() == T &&
              stride.numel() == T && base.is_contiguous() && stride.is_contiguous(), "match_rows: tables");
  TORCH_CHECK(meta.dtype() == torch::kInt64 && moff.dtype() == torch::kInt64 && moff.numel() == T &&
              meta.is_contiguous() && moff.is_contiguous(), "match_rows: meta tables");
  if ((int64_t)py::len(rows) != K) return false;
  const int64_t* B = base.data_ptr<int64_t>();
  const int64_t* S = stride.data_ptr<int64_t>();
  const int64_t* M = meta.data_ptr<int64_t>();
  const int64_t* MO = moff.data_ptr<int64_t>();
  for (int64_t i = 0; i < K; ++i) {
    PyObject* d = PyList_GET_ITEM(dicts.ptr(), i);
    if (!PyDict_Check(d) || PyDict_GET_SIZE(d) != T) return false;
    const int64_t row = PyLong_AsLongLong(PyList_GET_ITEM(rows.ptr(), i));
    if (row == -1 && PyErr_Occurred()) throw py::error_already_set();
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    for (int64_t t = 0; t < T; ++t) {
      if (!PyDict_Next(d, &pos, &k, &v)) return false;
      PyObject* want = PyList_GET_ITEM(keys.ptr(), t);
      if (k != want) {
        const int eq = PyObject_RichCompareBool(k, want, Py_EQ);
        if (eq < 0) throw py::error_already_set();
        if (!eq) return false;
      }
      if (!THPVariable_Check(v)) return false;
      const at::Tensor& x = THPVariable_Unpack(v);
      if ((int64_t)x.data_ptr() != B[t] + row * S[t] || !x.is_contiguous()) return false;
      const int64_t* m = M + MO[t];
      if ((int64_t)x.scalar_type() != m[0] || (int64_t)x.dim() != m[1]) return false;
      for (int64_t a = 0; a < m[1]; ++a)
        if (x.size(a) != m[2 + a]) return false;
    }
  }
  return true;
}

// small_host_round(dicts, keys, mode, coef, divisor, fn, err_fn, ctx, stream, max_bytes, cpu_max_bytes) ->
// OrderedDict | None: a whole small host-resident round (cfg1, the reference's quick_start: K = 2
// LR-MNIST dicts, 63 KB a client) in one call -- the walk of gather(), the CPU outputs of
// alloc_outputs() and one call of the C ABI's fa_weighted_sum_host per dtype group, through the
// function pointer `fn` (libfedagg.so, loaded by the binding), with the GIL released while it runs.
// The C ABI packs the inputs into its mapped pinned buffer, the device computes, the result is
// copied into the fresh CPU tensors returned here (never recycled: the caller owns them).  Returns
// None -- the general path then runs and raises the reference's errors -- unless every value is a
// contiguous CPU tensor of a C-ABI dtype, the clients agree on every key's dtype and shape, and the
// round's input bytes are <= max_bytes with K, T <= 4096 (fa_weighted_sum_host's table limits).
// Rounds of at most cpu_max_bytes input bytes are summed right here on the host instead
// (fa_host::sum_key_any, host_sum.h: the same ordered per-element arithmetic, bit for bit) -- the
// engine's measured break-even below which a PCIe round trip costs more than the sum itself.
using wsum_host_fn = int (*)(void*, int, int, int32_t, const int64_t*, int32_t, const void* const*, const double*,
                             double, void* const*, void*);
using last_error_fn = const char* (*)();

py::object small_host_round(py::list dicts, py::list keys, int mode, py::object coef, double divisor, int64_t fn,
                            int64_t err_fn, int64_t ctx, int64_t stream, int64_t max_bytes, int64_t cpu_max_bytes) {
  const int64_t K = (int64_t)py::len(dicts);
  const int64_t T = (int64_t)py::len(keys);
  if (K == 0 || T == 0 || K > 4096 || T > 4096) return py::none();
  std::vector<double> w((size_t)K, 0.0);
  if (mode != 2) {  // FA_MODE_SUM = 2: no coefficients
    if (coef.is_none() || (int64_t)py::len(coef) != K) return py::none();
    py::sequence cs = coef;
    for (int64_t i = 0; i < K; ++i) w[i] = cs[i].cast<double>();
  }
  std::vector<PyObject*> kv(T);
  for (int64_t t = 0; t < T; ++t) kv[t] = PyList_GET_ITEM(keys.ptr(), t);
  std::vector<int64_t> ptr((size_t)(T * K)), numel(T);
  std::vector<int> code(T);
  std::vector<at::ScalarType> st(T);
  std::vector<c10::IntArrayRef> shape(T);
  std::vector<at::Tensor> first(T);  // client 0's tensors (their sizes() stay valid while held)
  std::vector<at::Tensor> keep;       // every input, referenced while the GIL is released below
  keep.reserve((size_t)(K * T));
  int64_t in_bytes = 0;
  for (int64_t i = 0; i < K; ++i) {
    PyObject* d = PyList_GET_ITEM(dicts.ptr(), i);
    if (!PyDict_Check(d) || PyDict_GET_SIZE(d) != T) return py::none();
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    for (int64_t t = 0; t < T; ++t) {
      if (!PyDict_Next(d, &pos, &k, &v)) return py::none();
      if (k != kv[t]) {
        const int eq = PyObject_RichCompareBool(k, kv[t], Py_EQ);
        if (eq < 0) throw py::error_already_set();
        if (!eq) return py::none();
      }
      if (!THPVariable_Check(v)) return py::none();
      const at::Tensor& x = THPVariable_Unpack(v);
      if (!x.device().is_cpu() || !x.is_contiguous()) return py::none();
      if (i == 0) {
        st[t] = x.scalar_type();
        code[t] = fa_dtype_code(st[t]);
        if (code[t] < 0) return py::none();
        first[t] = x;
        shape[t] = first[t].sizes();
        numel[t] = x.numel();
        in_bytes += numel[t] * (int64_t)x.element_size() * K;
        if (in_bytes > max_bytes) return py::none();
      } else if (x.scalar_type() != st[t] || x.sizes() != shape[t]) {
        return py::none();
      }
      ptr[t * K + i] = (int64_t)x.data_ptr();
      keep.push_back(x);
    }
  }
  // outputs: one CPU allocation, every key on a 256-byte boundary; weighted modes turn int64 into
  // float32 (PyTorch's int64 * python float)
  std::vector<at::ScalarType> ost(T);
  std::vector<int64_t> off(T);
  int64_t total = 0;
  for (int64_t t = 0; t < T; ++t) {
    ost[t] = (code[t] == 4 && mode != 2) ? at::kFloat : st[t];
    off[t] = total;
    total += (numel[t] * (int64_t)c10::elementSize(ost[t]) + 255) / 256 * 256;
  }
  auto arena = torch::empty({std::max<int64_t>(total, 256)}, torch::TensorOptions().dtype(torch::kUInt8));
  char* base = (char*)arena.data_ptr();
  // one C-ABI call per dtype group (key-major tables, keys in their dict order within a group)
  int rc = 0;
  if (in_bytes <= cpu_max_bytes) {  // small host-resident round: summed where the data already is
    py::gil_scoped_release nogil;
    std::vector<const void*> in((size_t)K);
    for (int64_t t = 0; t < T && rc == 0; ++t) {
      for (int64_t i = 0; i < K; ++i) in[i] = (const void*)ptr[t * K + i];
      rc = fa_host::sum_key_any(code[t], mode, numel[t], (int)K, in.data(), mode == 2 ? nullptr : w.data(), divisor,
                                base + off[t]);
    }
    if (rc != 0) throw std::runtime_error("small_host_round: host sum rejected a dtype / mode");
  } else {
    py::gil_scoped_release nogil;
    std::vector<int64_t> gn, gin, gout;
    for (int c = 0; c <= 4 && rc == 0; ++c) {
      gn.clear();
      gin.clear();
      gout.clear();
      for (int64_t t = 0; t < T; ++t) {
        if (code[t] != c) continue;
        gn.push_back(numel[t]);
        for (int64_t i = 0; i < K; ++i) gin.push_back(ptr[t * K + i]);
        gout.push_back((int64_t)(base + off[t]));
      }
      if (gn.empty()) continue;
      rc = reinterpret_cast<wsum_host_fn>(fn)((void*)ctx, c, mode, (int32_t)gn.size(), gn.data(), (int32_t)K,
                                              reinterpret_cast<const void* const*>(gin.data()), w.data(), divisor,
                                              reinterpret_cast<void* const*>(gout.data()), (void*)stream);
    }
  }
  if (rc != 0)
    throw std::runtime_error(std::string("fa_weighted_sum_host failed (") + std::to_string(rc) +
                             "): " + reinterpret_cast<last_error_fn>(err_fn)());
  static PyObject* odict_type = [] {  // collections.OrderedDict, held for the process lifetime
    PyObject* mod = PyImport_ImportModule("collections");
    if (!mod) throw py::error_already_set();
    PyObject* t = PyObject_GetAttrString(mod, "OrderedDict");
    Py_DECREF(mod);
    if (!t) throw py::error_already_set();
    return t;
  }();
  py::object out = py::reinterpret_steal<py::object>(PyObject_CallNoArgs(odict_type));
  if (!out) throw py::error_already_set();
  const c10::Storage& storage = arena.storage();
  const c10::DispatchKeySet ks = arena.key_set();
  for (int64_t t = 0; t < T; ++t) {
    at::Tensor v = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(storage), ks,
                                                            caffe2::TypeMeta::fromScalarType(ost[t]));
    c10::TensorImpl* impl = v.unsafeGetTensorImpl();
    impl->set_storage_offset(off[t] / (int64_t)c10::elementSize(ost[t]));
    impl->set_sizes_contiguous(shape[t]);
    py::object pv = py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(v)));
    if (PyObject_SetItem(out.ptr(), kv[t], pv.ptr()) < 0) throw py::error_already_set();
  }
  return out;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("small_host_round", &small_host_round,
        "a whole small host-resident round: summed on the host below cpu_max_bytes, else through fa_weighted_sum_host",
        py::arg("dicts"), py::arg("keys"), py::arg("mode"), py::arg("coef"), py::arg("divisor"), py::arg("fn"),
        py::arg("err_fn"), py::arg("ctx"), py::arg("stream"), py::arg("max_bytes"), py::arg("cpu_max_bytes") = 0);
  m.def("match_rows", &match_rows, "are these state_dicts the row views of one arena?");
  m.def("pack_range", &pack_range, "multi-threaded packing of host tensors into a pinned staging range");
  m.doc() = "host-side table builder of the fedml_amd aggregation engine (no tensor data access)";
  m.def("gather", &gather, "validate K client dicts x T keys, return the device pointer table");
  m.def("carve", &carve, "contiguous views of a flat tensor at element offsets");
  m.def("alloc_outputs", &alloc_outputs, "carve T aligned outputs out of one device allocation");
  m.def("plan_outputs", &plan_outputs, "outputs of a device round plus its per-dtype launch tables");
}
