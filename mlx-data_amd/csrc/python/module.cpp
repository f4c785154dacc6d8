// module.cpp -- pybind11 binding of the pipeline (csrc/pipeline) with the
// mlx.data Python surface for the image path: names and keyword arguments of
// python/src/wrap_dataset.h:83-110,305-332,364-402,746-777,
// wrap_stream.cpp:123-129,340-377, wrap_buffer.cpp:93,250,342,358,373 and
// the numpy conversions of wrap.cpp:27-222.  The GIL is released around every
// get()/next(), so prefetch workers (and the GPU launches they issue) run in
// parallel; Python callbacks (key_transform functions, the image decoder)
// re-acquire it.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <sstream>

#include "../pipeline/pipeline.h"
#include "mxd_amd.h"

namespace py = pybind11;
using namespace mxd::pipe;

namespace {

// ------------------------------------------------------------ numpy -> Array
std::shared_ptr<Array> to_array(py::handle obj);

std::shared_ptr<Array> from_numpy(py::array a) {
  if (!(a.flags() & py::detail::npy_api::constants::NPY_ARRAY_C_CONTIGUOUS_))
    throw std::runtime_error("[to_array] Contiguous array expected -- use numpy.ascontiguousarray()");
  std::vector<int64_t> shape(a.ndim());
  for (int i = 0; i < a.ndim(); i++) shape[i] = a.shape(i);
  // Zero copy: the Array keeps a reference to the numpy object, dropped under
  // the GIL (wrap.cpp:97-105).  Read-only arrays are fine: the pipeline never
  // writes into an input.
  auto handle = a.inc_ref();
  std::shared_ptr<void> data(const_cast<void*>(a.data()), [handle](void*) {
    py::gil_scoped_acquire gil;
    handle.dec_ref();
  });
  DType t;
  switch (a.dtype().char_()) {
    case 'f': t = DType::Float; break;
    case 'd': t = DType::Double; break;
    case 'i': t = DType::Int32; break;
    case 'l':
    case 'q': t = DType::Int64; break;
    case 'b': t = DType::Int8; break;
    case 'B': t = DType::UInt8; break;
    case 'S':
      shape.push_back(a.itemsize());
      t = DType::Int8;
      break;
    default: {
      std::ostringstream msg;
      msg << "[to_array] Unsupported array type '" << a.dtype().char_() << "'";
      throw std::invalid_argument(msg.str());
    }
  }
  return std::make_shared<Array>(t, shape, data);
}

std::shared_ptr<Array> scalar_i64(int64_t v) {
  auto buf = std::shared_ptr<void>(new int64_t(v), [](void* p) { delete static_cast<int64_t*>(p); });
  return std::make_shared<Array>(DType::Int64, std::vector<int64_t>{}, buf);
}

std::shared_ptr<Array> scalar_f64(double v) {
  auto buf = std::shared_ptr<void>(new double(v), [](void* p) { delete static_cast<double*>(p); });
  return std::make_shared<Array>(DType::Double, std::vector<int64_t>{}, buf);
}

std::shared_ptr<Array> from_bytes(const char* p, size_t n) {
  auto a = std::make_shared<Array>(DType::Int8, std::vector<int64_t>{(int64_t)n});
  if (n) std::memcpy(a->data(), p, n);
  return a;
}

struct DeviceArray;
std::shared_ptr<Array> device_array_of(py::handle obj);

std::shared_ptr<Array> to_array(py::handle obj) {
  if (py::isinstance<py::array>(obj)) return from_numpy(obj.cast<py::array>());
  if (auto d = device_array_of(obj)) return d;
  if (py::isinstance<py::bool_>(obj) || py::isinstance<py::int_>(obj)) return scalar_i64(obj.cast<int64_t>());
  if (py::isinstance<py::float_>(obj)) return scalar_f64(obj.cast<double>());
  if (py::isinstance<py::bytes>(obj)) {
    char* p;
    Py_ssize_t n;
    PyBytes_AsStringAndSize(obj.ptr(), &p, &n);
    return from_bytes(p, (size_t)n);
  }
  if (py::isinstance<py::str>(obj))
    throw std::invalid_argument("[to_array] Cannot convert strings to arrays. Please encode them as bytes first.");
  // A Python buffer (bytearray, array.array, memoryview ...) is copied: it
  // may be mutable and is not ours to alias (wrap.cpp:159-163, to_array(py::buffer)).
  if (py::isinstance<py::buffer>(obj)) {
    py::buffer_info info = obj.cast<py::buffer>().request();
    int64_t expect = info.itemsize;
    bool contiguous = true;
    for (int d = info.ndim - 1; d >= 0; d--) {
      if (info.shape[d] > 1 && info.strides[d] != expect) contiguous = false;
      expect *= info.shape[d];
    }
    if (!contiguous) throw std::invalid_argument("[to_array] Contiguous buffer expected -- maybe cast to np.array");
    py::array a = py::array::ensure(obj);
    if (!a) throw std::invalid_argument("[to_array] Unsupported buffer type '" + info.format + "'");
    return from_numpy(a.attr("copy")().cast<py::array>());
  }
  // Anything else with the array interface (wrap.cpp:165-175).
  try {
    return from_numpy(py::array::ensure(obj));
  } catch (const std::exception&) {
  }
  std::ostringstream msg;
  msg << "[to_array] Cannot convert type " << py::str(py::type::of(obj)).cast<std::string>()
      << " to an array. Use a numpy array, a python buffer or scalar.";
  throw std::invalid_argument(msg.str());
}

// ------------------------------------------------------------ Array -> numpy
py::dtype np_dtype(DType t) {
  switch (t) {
    case DType::Int8: return py::dtype("b");
    case DType::UInt8: return py::dtype("B");
    case DType::Int32: return py::dtype("i4");
    case DType::Int64: return py::dtype("i8");
    case DType::Float: return py::dtype("f");
    case DType::Double: return py::dtype("d");
    default: throw std::runtime_error("internal error: unknown type");
  }
}

py::array to_numpy(const std::shared_ptr<Array>& a) {
  void* data;
  {
    // May run the pending GPU work of this array.
    py::gil_scoped_release nogil;
    data = a->data();
  }
  py::dtype dt = np_dtype(a->type());
  auto* keep = new std::shared_ptr<Array>(a);
  py::capsule owner(keep, [](void* p) { delete static_cast<std::shared_ptr<Array>*>(p); });
  std::vector<int64_t> shape = a->shape(), strides(shape.size());
  int64_t s = itemsize(a->type());
  for (int d = (int)shape.size() - 1; d >= 0; d--) {
    strides[d] = s;
    s *= shape[d];
  }
  return py::array(dt, shape, strides, data, owner);
}

// ------------------------------------------------------------ device arrays
// DLPack (v0.8 ABI, dlpack.h): a device batch is handed to consumers
// (torch.from_dlpack, ...) without a copy.  Only the layout is restated here.
struct DLDevice {
  int32_t device_type;  // kDLROCM = 10
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;  // kDLInt 0, kDLUInt 1, kDLFloat 2
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;

DLDataType dl_dtype(DType t) {
  switch (t) {
    case DType::UInt8: return {1, 8, 1};
    case DType::Int8: return {0, 8, 1};
    case DType::Int32: return {0, 32, 1};
    case DType::Int64: return {0, 64, 1};
    case DType::Float: return {2, 32, 1};
    case DType::Double: return {2, 64, 1};
    default: throw std::runtime_error("internal error: unknown type");
  }
}

// The Python face of a device-resident Array.
struct DeviceArray {
  std::shared_ptr<Array> a;
};

struct DLHolder {
  std::shared_ptr<Array> a;
  std::vector<int64_t> shape;
  DLManagedTensor t{};
};

py::capsule to_dlpack(const std::shared_ptr<Array>& a) {
  auto* h = new DLHolder{a, a->shape(), {}};
  h->t.dl_tensor.data = a->data();
  h->t.dl_tensor.device = {kDLROCM, a->device()};
  h->t.dl_tensor.ndim = a->ndim();
  h->t.dl_tensor.dtype = dl_dtype(a->type());
  h->t.dl_tensor.shape = h->shape.data();
  h->t.dl_tensor.strides = nullptr;  // compact row-major
  h->t.manager_ctx = h;
  h->t.deleter = [](DLManagedTensor* t) { delete static_cast<DLHolder*>(t->manager_ctx); };
  // A capsule never consumed ("dltensor" still its name) frees the tensor.
  return py::capsule(&h->t, "dltensor", [](PyObject* cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (t && t->deleter) t->deleter(t);
    }
  });
}

py::array device_to_numpy(const std::shared_ptr<Array>& a) {
  py::array host = to_numpy(std::make_shared<Array>(a->type(), a->shape()));
  {
    py::gil_scoped_release nogil;
    if (a->nbytes() > 0 && mxd_memcpy_d2h(host.mutable_data(), a->data(), (size_t)a->nbytes(), a->device()) != MXD_OK)
      throw std::runtime_error(mxd_last_error());
  }
  return host;
}

py::object to_py(const std::shared_ptr<Array>& a) {
  if (a->device() >= 0) return py::cast(DeviceArray{a});
  return to_numpy(a);
}

py::dict to_dict(const Sample& s) {
  py::dict d;
  for (const auto& kv : s) d[py::str(kv.first)] = to_py(kv.second);
  return d;
}

Sample to_sample(py::handle obj) {
  if (!py::isinstance<py::dict>(obj)) throw std::invalid_argument("Sample: dict expected");
  Sample s;
  for (auto kv : obj.cast<py::dict>()) s[kv.first.cast<std::string>()] = to_array(kv.second);
  return s;
}

// A Python callable that may be destroyed from a worker thread.
std::shared_ptr<py::function> hold(py::function f) {
  return std::shared_ptr<py::function>(new py::function(std::move(f)), [](py::function* p) {
    if (_Py_IsFinalizing()) return;  // the interpreter is going: taking the GIL would block forever
    py::gil_scoped_acquire gil;
    delete p;
  });
}

// A prefetching stream or buffer whose last Python reference goes away joins
// its worker threads, and those may be waiting for the GIL (a Python
// key_transform, the image decoder): destroy it with the GIL released.  At
// interpreter exit the workers can no longer take the GIL at all, so the
// object is left to the process teardown.
template <class T>
std::shared_ptr<T> nogil_owned(T* obj) {
  return std::shared_ptr<T>(obj, [](T* o) {
    if (_Py_IsFinalizing()) return;
    if (PyGILState_Check()) {
      py::gil_scoped_release nogil;
      delete o;
    } else {
      delete o;
    }
  });
}

// ------------------------------------------------------------ dataset ops
// The ops every Dataset (Buffer and Stream) carries (wrap_dataset.h).
template <class D, class Wrap>
void dataset_ops(py::class_<D, std::shared_ptr<D>>& cls, Wrap wrap) {
  using Self = std::shared_ptr<D>;
  cls.def(
         "key_transform",
         [wrap](const Self& self, const std::string& key, py::function func, const std::string& output_key) {
           auto fn = hold(std::move(func));
           auto op = std::make_shared<KeyTransform>(
               key,
               [fn](const std::shared_ptr<Array>& x) {
                 py::gil_scoped_acquire gil;
                 return to_array((*fn)(to_py(x)));
               },
               output_key);
           return wrap(self, op);
         },
         py::arg("key"), py::arg("func"), py::arg("output_key") = "")
      .def(
          "load_image",
          [wrap](const Self& self, const std::string& key, const std::string& prefix, bool info,
                 const std::string& format, bool from_memory, const std::string& output_key) {
            return wrap(self, std::make_shared<LoadImage>(key, prefix, info, format, from_memory, output_key));
          },
          py::arg("key"), py::arg("prefix") = "", py::arg("info") = false, py::arg("format") = "RGB",
          py::arg("from_memory") = false, py::arg("output_key") = "")
      .def(
          "image_resize_smallest_side",
          [wrap](const Self& self, const std::string& key, int64_t size, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageResizeSmallestSide>(key, size, output_key));
          },
          py::arg("key"), py::arg("size"), py::arg("output_key") = "")
      .def(
          "image_resize",
          [wrap](const Self& self, const std::string& key, int64_t w, int64_t h, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageResize>(key, w, h, output_key));
          },
          py::arg("key"), py::arg("w"), py::arg("h"), py::arg("output_key") = "")
      .def(
          "image_center_crop",
          [wrap](const Self& self, const std::string& key, int64_t w, int64_t h, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageCenterCrop>(key, w, h, output_key));
          },
          py::arg("key"), py::arg("w"), py::arg("h"), py::arg("output_key") = "")
      .def(
          "image_random_crop",
          [wrap](const Self& self, const std::string& key, int64_t w, int64_t h, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageRandomCrop>(key, w, h, output_key));
          },
          py::arg("key"), py::arg("w"), py::arg("h"), py::arg("output_key") = "")
      .def(
          "image_random_h_flip",
          [wrap](const Self& self, const std::string& key, float prob, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageRandomHFlip>(key, prob, output_key));
          },
          py::arg("key"), py::arg("prob"), py::arg("output_key") = "")
      .def(
          "image_random_area_crop",
          [wrap](const Self& self, const std::string& key, std::pair<float, float> area_range,
                 std::pair<float, float> aspect_ratio_range, int num_trial, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageRandomAreaCrop>(key, area_range, aspect_ratio_range, num_trial,
                                                                    output_key));
          },
          py::arg("key"), py::arg("area_range"), py::arg("aspect_ratio_range"), py::arg("num_trial") = 10,
          py::arg("output_key") = "")
      .def(
          "image_rotate",
          [wrap](const Self& self, const std::string& key, double angle, bool crop, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageRotate>(key, angle, crop, output_key));
          },
          py::arg("key"), py::arg("angle"), py::arg("crop") = false, py::arg("output_key") = "")
      .def(
          "image_channel_reduction",
          [wrap](const Self& self, const std::string& key, const std::string& preset, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageChannelReduction>(key, preset, output_key));
          },
          py::arg("key"), py::arg("preset") = "default", py::arg("output_key") = "")
      .def(
          "image_to_float",
          [wrap](const Self& self, const std::string& key, const std::string& output_key) {
            return wrap(self, std::make_shared<ImageToFloat>(key, output_key));
          },
          py::arg("key"), py::arg("output_key") = "");
}

using PadMap = std::unordered_map<std::string, double>;
using DimMap = std::unordered_map<std::string, int>;

std::shared_ptr<Array> device_array_of(py::handle obj) {
  if (!py::isinstance<DeviceArray>(obj)) return nullptr;
  return obj.cast<const DeviceArray&>().a;
}

// batch(..., device=None | int, device_keys=None | [str])
DeviceOut device_out(const py::object& device, const py::object& keys) {
  DeviceOut o;
  if (!device.is_none()) {
    o.device = device.cast<int>();
    if (o.device < 0) throw std::invalid_argument("batch: device must be a device index >= 0");
  }
  if (!keys.is_none()) o.keys = keys.cast<std::vector<std::string>>();
  if (!o.keys.empty() && o.device < 0) throw std::invalid_argument("batch: device_keys needs device");
  return o;
}

}  // namespace

PYBIND11_MODULE(_pipeline, m) {
  m.doc() = "mlx.data image-path operator surface over the gfx950 resize/crop kernels";

  py::class_<DeviceArray>(m, "DeviceArray",
                          "A batch tensor in device memory (batch(..., device=d)): DLPack producer "
                          "(__dlpack__ / __dlpack_device__, kDLROCM), numpy() copies it to the host.")
      .def_property_readonly("shape", [](const DeviceArray& d) { return py::tuple(py::cast(d.a->shape())); })
      .def_property_readonly("dtype", [](const DeviceArray& d) { return np_dtype(d.a->type()); })
      .def_property_readonly("device", [](const DeviceArray& d) { return d.a->device(); })
      .def_property_readonly("data_ptr", [](const DeviceArray& d) { return reinterpret_cast<uintptr_t>(d.a->data()); })
      .def_property_readonly("nbytes", [](const DeviceArray& d) { return d.a->nbytes(); })
      .def("__dlpack__", [](const DeviceArray& d, py::kwargs) { return to_dlpack(d.a); })
      .def("__dlpack_device__", [](const DeviceArray& d) { return py::make_tuple(kDLROCM, d.a->device()); })
      .def("numpy", [](const DeviceArray& d) { return device_to_numpy(d.a); })
      .def("__array__", [](const DeviceArray& d, py::args, py::kwargs) { return device_to_numpy(d.a); })
      .def("__len__", [](const DeviceArray& d) { return d.a->ndim() ? d.a->shape(0) : 0; })
      .def("__repr__", [](const DeviceArray& d) {
        std::ostringstream o;
        o << "DeviceArray(shape=(";
        for (int i = 0; i < d.a->ndim(); i++) o << (i ? ", " : "") << d.a->shape(i);
        o << (d.a->ndim() == 1 ? ",)" : ")") << ", device=" << d.a->device() << ")";
        return o.str();
      });

  py::class_<Buffer, std::shared_ptr<Buffer>> buffer(m, "Buffer");
  py::class_<Stream, std::shared_ptr<Stream>> stream(m, "Stream");

  dataset_ops(buffer, [](const std::shared_ptr<Buffer>& b, std::shared_ptr<Op> op) -> std::shared_ptr<Buffer> {
    return std::make_shared<BufferTransform>(b, std::move(op));
  });
  dataset_ops(stream, [](const std::shared_ptr<Stream>& s, std::shared_ptr<Op> op) -> std::shared_ptr<Stream> {
    return std::make_shared<StreamTransform>(s, std::move(op));
  });

  buffer.def("size", &Buffer::size)
      .def("__len__", &Buffer::size)
      .def("__getitem__",
           [](const std::shared_ptr<Buffer>& b, int64_t idx) {
             Sample s;
             {
               py::gil_scoped_release nogil;
               idx = idx < 0 ? idx + b->size() : idx;  // wrap_buffer.cpp:62
               s = b->get(idx);
             }
             return to_dict(s);
           })
      .def("shuffle", [](const std::shared_ptr<Buffer>& b) { return shuffle_buffer(b); })
      .def("perm",
           [](const std::shared_ptr<Buffer>& b, std::vector<int64_t> perm) -> std::shared_ptr<Buffer> {
             return std::make_shared<Perm>(b, std::move(perm));
           })
      .def("to_stream", [](const std::shared_ptr<Buffer>& b) -> std::shared_ptr<Stream> {
        return std::make_shared<FromBuffer>(b);
      })
      .def(
          "batch",
          [](const std::shared_ptr<Buffer>& b, int64_t batch_size, PadMap pad, DimMap dim, py::object device,
             py::object device_keys) -> std::shared_ptr<Buffer> {
            return std::make_shared<BufferBatch>(b, batch_size, std::move(pad), std::move(dim),
                                                 device_out(device, device_keys));
          },
          py::arg("batch_size"), py::arg("pad") = PadMap{}, py::arg("dim") = DimMap{}, py::arg("device") = py::none(),
          py::arg("device_keys") = py::none())
      .def(
          "ordered_prefetch",
          [](const std::shared_ptr<Buffer>& b, int prefetch_size, int num_threads) -> std::shared_ptr<Stream> {
            return nogil_owned<Stream>(new OrderedPrefetch(b, prefetch_size, num_threads));
          },
          py::arg("prefetch_size"), py::arg("num_threads"));

  stream
      .def("next",
           [](const std::shared_ptr<Stream>& s) {
             Sample x;
             {
               py::gil_scoped_release nogil;
               x = s->next();
             }
             return to_dict(x);
           })
      .def("reset",
           [](const std::shared_ptr<Stream>& s) {
             py::gil_scoped_release nogil;
             s->reset();
           })
      .def(
          "batch",
          [](const std::shared_ptr<Stream>& s, int64_t batch_size, PadMap pad, DimMap dim, py::object device,
             py::object device_keys) -> std::shared_ptr<Stream> {
            return std::make_shared<StreamBatch>(s, batch_size, std::move(pad), std::move(dim),
                                                 device_out(device, device_keys));
          },
          py::arg("batch_size"), py::arg("pad") = PadMap{}, py::arg("dim") = DimMap{}, py::arg("device") = py::none(),
          py::arg("device_keys") = py::none())
      .def(
          "prefetch",
          [](const std::shared_ptr<Stream>& s, int prefetch_size, int num_threads) -> std::shared_ptr<Stream> {
            return nogil_owned<Stream>(new Prefetch(s, prefetch_size, num_threads));
          },
          py::arg("prefetch_size"), py::arg("num_threads"));

  m.def("buffer_from_vector", [](py::list data) -> std::shared_ptr<Buffer> {
    std::vector<Sample> samples;
    samples.reserve(data.size());
    for (auto item : data) {
      samples.push_back(to_sample(item));
      if (samples.back().empty()) throw std::runtime_error("FromVector: unexpected empty sample");
    }
    return std::make_shared<FromVector>(std::move(samples));
  });

  m.def("set_state", &set_state, py::arg("seed") = 1234);
  m.def("set_devices", &set_devices, py::arg("devices"));
  // diagnostics: how a batch of n images is split over ndev devices
  m.def(
      "_split_batch",
      [](int64_t n, int64_t ndev, uint64_t first) {
        std::vector<std::tuple<int64_t, int64_t, int64_t>> out;
        for (const Slice& s : split_batch(n, ndev, first)) out.emplace_back(s.device, s.begin, s.end);
        return out;
      },
      py::arg("n"), py::arg("ndev"), py::arg("first") = 0);
  m.attr("_MIN_SLICE_IMAGES") = kMinSliceImages;
  m.def("devices", &devices);
  m.def("set_device_decode", &set_device_decode, py::arg("on"));
  m.def("set_device_entropy", &set_device_entropy, py::arg("on"));
  m.def("device_entropy", &device_entropy);
  m.def("device_decode", &device_decode);
  m.def("_device_pool_bytes", &device_pool_bytes, py::arg("device"));
  m.def("_run_on_stats", &run_on_stats, py::arg("reset") = false);
  m.def("_pipe_stats", &pipe_stats, py::arg("reset") = false);

  // The decoder holds a Python callable: drop it before the interpreter goes.
  py::module_::import("atexit").attr("register")(py::cpp_function([] { set_image_decoder(nullptr); }));

  // fn(path: str, data: numpy int8 | None, from_memory: bool, info: bool)
  //   -> uint8 (H, W, C) array, (w, h) for info, or None.
  m.def("set_image_decoder", [](py::function fn) {
    auto f = hold(std::move(fn));
    set_image_decoder([f](const std::string& path, const std::shared_ptr<Array>& bytes, bool from_memory,
                          bool info) -> std::shared_ptr<Array> {
      py::gil_scoped_acquire gil;
      py::object data = from_memory ? py::object(to_numpy(bytes)) : py::object(py::none());
      py::object r = (*f)(path, data, from_memory, info);
      if (r.is_none()) return nullptr;
      return to_array(r);
    });
  });

  // Test hooks: whether a sample value is still a pending GPU plan.
  m.def("_pending", [](const std::shared_ptr<Buffer>& b, int64_t idx, const std::string& key) {
    Sample s;
    {
      py::gil_scoped_release nogil;
      s = b->get(idx);
    }
    return check_key(s, key)->pending();
  });
  m.def("_plan", [](const std::shared_ptr<Buffer>& b, int64_t idx, const std::string& key) -> py::object {
    Sample s;
    {
      py::gil_scoped_release nogil;
      s = b->get(idx);
    }
    auto a = check_key(s, key);
    if (!a->pending()) return py::none();
    const ImagePlan& p = *a->plan();
    py::dict d;
    d["src_shape"] = p.src->shape();
    d["window"] = py::make_tuple(p.sx, p.sy, p.sw, p.sh);
    d["resize"] = py::make_tuple(p.resize_w, p.resize_h);
    d["crop"] = py::make_tuple(p.crop_x, p.crop_y, p.crop_w, p.crop_h);
    d["flip"] = p.flip;
    d["shape"] = a->shape();
    return d;
  });
}
