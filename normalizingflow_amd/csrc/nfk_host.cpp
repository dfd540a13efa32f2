// nfk_host.cpp -- host-side cache validation for the layers with thousands of
// parameter tensors (CPython extension, CPU only; no device work).
//
// A fused layer's weight pack is valid while every parameter keeps its storage
// and version counter and the conditioner modules are the same objects
// (normalizingflow_amd/flows.py: the caches are keyed on exactly that).  At
// Polymer.yaml's NSF_AR (applications/input/Polymer.yaml: 2,047 conditioners,
// 6,142 parameter tensors per layer) computing that key in Python took ~23 ms
// per call -- forty times the layer's kernel.  ar_state() walks the same module
// tree in C++ (~1 ms) and returns a 64-bit hash of it, or -1 when a
// conditioner is not the stock FCNN (flows.py:20-35).  ar_watch() walks it
// once and keeps what the key depends on: every dict on the way (CPython's
// per-dict version tag, PEP 509, changes with any insertion, deletion or
// replacement) and every parameter (storage pointer, version counter); its
// valid() then compares ~10 K cached words (~20 us at Polymer) instead of
// re-walking the tree.
#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/utils/pybind.h>

#include <cstdint>
#include <memory>
#include <vector>

namespace {

struct Hash {
    uint64_t h = 1469598103934665603ull;
    void mix(uint64_t v) {
        h = (h ^ v) * 1099511628211ull;
        h ^= h >> 29;
    }
};

// interned keys (PyDict_GetItemString would build a string object per lookup)
struct Keys {
    PyObject *modules, *network, *parameters, *weight, *bias;
    Keys()
        : modules(PyUnicode_InternFromString("_modules")), network(PyUnicode_InternFromString("network")),
          parameters(PyUnicode_InternFromString("_parameters")), weight(PyUnicode_InternFromString("weight")),
          bias(PyUnicode_InternFromString("bias")) {}
};
const Keys& keys() {
    static const Keys k;
    return k;
}

PyObject* inst_dict_item(PyObject* obj, PyObject* key) {
    PyObject** dp = _PyObject_GetDictPtr(obj);
    if (dp == nullptr || *dp == nullptr) return nullptr;
    return PyDict_GetItem(*dp, key);  // borrowed
}

bool mix_tensor(Hash& h, PyObject* t) {
    if (t == nullptr || !THPVariable_Check(t)) return false;
    const at::Tensor& v = THPVariable_Unpack(t);
    h.mix((uint64_t)(uintptr_t)v.unsafeGetTensorImpl()->data());
    h.mix((uint64_t)v._version());
    return true;
}

// (data_ptr, version) of every tensor of a list
int64_t fingerprint(py::list ts) {
    Hash h;
    for (py::handle o : ts)
        if (!mix_tensor(h, o.ptr())) throw py::type_error("fingerprint: not a tensor");
    return (int64_t)h.h;
}

// NSF_AR's conditioner tree: layers._modules (an ordered dict of FCNN), each
// FCNN's network._modules = {Linear, Tanh, Linear, Tanh, Linear}; the hash of
// every module's identity and every Linear's (weight, bias) state, plus
// init_param's; -1 when the tree is not that shape
int64_t ar_state(py::handle layers_modules, py::handle init_param, py::handle fcnn_t, py::handle linear_t,
                 py::handle tanh_t) {
    Hash h;
    if (!mix_tensor(h, init_param.ptr())) return -1;
    PyObject* d = layers_modules.ptr();
    if (!PyDict_Check(d)) return -1;
    PyObject *key, *cond;
    Py_ssize_t pos = 0;
    PyTypeObject* lin = (PyTypeObject*)linear_t.ptr();
    PyTypeObject* tnh = (PyTypeObject*)tanh_t.ptr();
    while (PyDict_Next(d, &pos, &key, &cond)) {
        if ((PyObject*)Py_TYPE(cond) != fcnn_t.ptr()) return -1;
        h.mix((uint64_t)(uintptr_t)cond);
        const Keys& K = keys();
        PyObject* cm = inst_dict_item(cond, K.modules);
        PyObject* net = (cm != nullptr && PyDict_Check(cm)) ? PyDict_GetItem(cm, K.network) : nullptr;
        if (net == nullptr) return -1;
        h.mix((uint64_t)(uintptr_t)net);
        PyObject* nm = inst_dict_item(net, K.modules);
        if (nm == nullptr || !PyDict_Check(nm) || PyDict_Size(nm) != 5) return -1;
        PyObject *k2, *sub;
        Py_ssize_t p2 = 0;
        int idx = 0;
        while (PyDict_Next(nm, &p2, &k2, &sub)) {
            const bool want_lin = (idx % 2) == 0;
            if (!PyObject_TypeCheck(sub, want_lin ? lin : tnh)) return -1;
            h.mix((uint64_t)(uintptr_t)sub);
            if (want_lin) {
                PyObject* pm = inst_dict_item(sub, K.parameters);
                if (pm == nullptr || !PyDict_Check(pm)) return -1;
                if (!mix_tensor(h, PyDict_GetItem(pm, K.weight))) return -1;
                if (!mix_tensor(h, PyDict_GetItem(pm, K.bias))) return -1;
            }
            ++idx;
        }
    }
    return (int64_t)(h.h & 0x7fffffffffffffffull);  // (never -1)
}

// (PEP 509's ma_version_tag: CPython 3.6-3.11; later versions deprecate it,
// and ar_watch() returns None there -- the caller falls back to ar_state)
#if PY_VERSION_HEX >= 0x03060000 && PY_VERSION_HEX < 0x030C0000
#define NFK_DICT_TAGS 1
#else
#define NFK_DICT_TAGS 0
#endif

class ArWatch {
   public:
    ArWatch() = default;
    ArWatch(const ArWatch&) = delete;
    ArWatch& operator=(const ArWatch&) = delete;
    ~ArWatch() {
        for (PyObject* o : dicts_) Py_DECREF(o);
        for (PyObject* o : tens_) Py_DECREF(o);
    }
    bool add_dict(PyObject* d) {
        if (d == nullptr || !PyDict_Check(d)) return false;
        Py_INCREF(d);
        dicts_.push_back(d);
        tags_.push_back(tag(d));
        return true;
    }
    bool add_tensor(PyObject* t) {
        if (t == nullptr || !THPVariable_Check(t)) return false;
        Py_INCREF(t);
        tens_.push_back(t);
        const at::Tensor& v = THPVariable_Unpack(t);
        ptrs_.push_back(storage_of(v));
        offs_.push_back(v.unsafeGetTensorImpl()->storage_offset());
        vers_.push_back(v._version());
        return true;
    }
    bool valid() const {
        for (size_t i = 0; i < dicts_.size(); ++i)
            if (tag(dicts_[i]) != tags_[i]) return false;
        for (size_t i = 0; i < tens_.size(); ++i) {
            const at::Tensor& v = THPVariable_Unpack(tens_[i]);
            if (v._version() != vers_[i] || storage_of(v) != ptrs_[i] ||
                v.unsafeGetTensorImpl()->storage_offset() != offs_[i])
                return false;
        }
        return true;
    }
    size_t size() const { return dicts_.size() + tens_.size(); }

   private:
    // (the storage's data pointer: TensorImpl::data() re-checks the storage
    // on every call and took ~30 ns per tensor)
    static const void* storage_of(const at::Tensor& v) {
        return v.unsafeGetTensorImpl()->unsafe_storage().unsafeGetStorageImpl()->data_ptr().get();
    }
    static uint64_t tag(PyObject* d) {
#if NFK_DICT_TAGS
        return reinterpret_cast<PyDictObject*>(d)->ma_version_tag;
#else
        (void)d;
        return 0;
#endif
    }
    std::vector<PyObject*> dicts_, tens_;
    std::vector<uint64_t> tags_;
    std::vector<const void*> ptrs_;
    std::vector<int64_t> offs_;
    std::vector<uint32_t> vers_;
};

// the watch of an NSF_AR layer: its own _parameters and _modules dicts (the
// latter holds `layers`: assigning a new ModuleList changes only it), init_param,
// and ar_state's tree (the same stock-shape checks); None when the tree is not
// that shape or the interpreter has no dict version tags
py::object ar_watch(py::handle layer_params, py::handle layer_modules, py::handle layers_modules,
                    py::handle init_param, py::handle fcnn_t, py::handle linear_t, py::handle tanh_t) {
    if (!NFK_DICT_TAGS) return py::none();
    auto w = std::make_unique<ArWatch>();
    if (!w->add_dict(layer_params.ptr()) || !w->add_dict(layer_modules.ptr()) || !w->add_tensor(init_param.ptr()))
        return py::none();
    PyObject* d = layers_modules.ptr();
    if (!w->add_dict(d)) return py::none();
    PyObject *key, *cond;
    Py_ssize_t pos = 0;
    PyTypeObject* lin = (PyTypeObject*)linear_t.ptr();
    PyTypeObject* tnh = (PyTypeObject*)tanh_t.ptr();
    const Keys& K = keys();
    while (PyDict_Next(d, &pos, &key, &cond)) {
        if ((PyObject*)Py_TYPE(cond) != fcnn_t.ptr()) return py::none();
        PyObject* cm = inst_dict_item(cond, K.modules);
        if (!w->add_dict(cm)) return py::none();
        PyObject* net = PyDict_GetItem(cm, K.network);
        if (net == nullptr) return py::none();
        PyObject* nm = inst_dict_item(net, K.modules);
        if (!w->add_dict(nm) || PyDict_Size(nm) != 5) return py::none();
        PyObject *k2, *sub;
        Py_ssize_t p2 = 0;
        int idx = 0;
        while (PyDict_Next(nm, &p2, &k2, &sub)) {
            const bool want_lin = (idx % 2) == 0;
            if (!PyObject_TypeCheck(sub, want_lin ? lin : tnh)) return py::none();
            if (want_lin) {
                PyObject* pm = inst_dict_item(sub, K.parameters);
                if (!w->add_dict(pm)) return py::none();
                if (!w->add_tensor(PyDict_GetItem(pm, K.weight))) return py::none();
                if (!w->add_tensor(PyDict_GetItem(pm, K.bias))) return py::none();
            }
            ++idx;
        }
    }
    return py::cast(w.release(), py::return_value_policy::take_ownership);
}

// a watch over given dicts (version tags) and tensors (storage, offset,
// version): e.g. a RealNVP layer's module tree and its 24 Linear tensors
// (flows.RealNVP._wide_pack); None without dict version tags
py::object make_watch(py::list dicts, py::list tensors) {
    if (!NFK_DICT_TAGS) return py::none();
    auto w = std::make_unique<ArWatch>();
    for (py::handle d : dicts)
        if (!w->add_dict(d.ptr())) throw py::type_error("make_watch: not a dict");
    for (py::handle t : tensors)
        if (!w->add_tensor(t.ptr())) throw py::type_error("make_watch: not a tensor");
    return py::cast(w.release(), py::return_value_policy::take_ownership);
}

}  // namespace

PYBIND11_MODULE(_nfk_host, m) {
    m.def("fingerprint", &fingerprint);
    m.def("ar_state", &ar_state);
    py::class_<ArWatch>(m, "ArWatch").def("valid", &ArWatch::valid).def("__len__", &ArWatch::size);
    m.def("ar_watch", &ar_watch);
    m.def("make_watch", &make_watch);
}
