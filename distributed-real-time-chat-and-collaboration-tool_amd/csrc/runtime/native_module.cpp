// pybind11 module `_native`: the CPU runtime pieces of drtc_amd.
//   * BlockAllocator  - paged-KV block free list with refcounts (engine)
//   * bcrypt_*        - password hashing for the auth service (GIL released:
//                       a cost-12 hash is ~0.25 s and must not stall the
//                       gRPC server's other threads)
//   * LogStore        - append-only, CRC-checked Raft log segments
//   * WordTokenizer   - chat tokenizer encode / decode for ASCII text (GIL released)
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bcrypt.h"
#include "block_allocator.h"
#include "log_store.h"
#include "tokenizer.h"

namespace py = pybind11;

PYBIND11_MODULE(_native, m) {
  m.doc() = "drtc_amd native CPU runtime";

  py::class_<drtc::BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int32_t, int32_t>(), py::arg("num_blocks"), py::arg("reserved") = 0)
      .def_property_readonly("num_blocks", &drtc::BlockAllocator::num_blocks)
      .def_property_readonly("num_free", &drtc::BlockAllocator::num_free)
      .def_property_readonly("num_used", &drtc::BlockAllocator::num_used)
      .def("can_allocate", &drtc::BlockAllocator::can_allocate)
      .def("allocate", &drtc::BlockAllocator::allocate)
      .def("allocate_one", &drtc::BlockAllocator::allocate_one)
      .def("incref", &drtc::BlockAllocator::incref)
      .def("free", &drtc::BlockAllocator::free)
      .def("refcount", &drtc::BlockAllocator::refcount);

  m.def("bcrypt_hashpw",
        [](py::bytes password, py::bytes salt) {
          std::string p = password, s = salt, out;
          {
            py::gil_scoped_release nogil;
            out = drtc::bcrypt_hashpw(p, s);
          }
          return py::bytes(out);
        },
        py::arg("password"), py::arg("salt"));
  m.def("bcrypt_checkpw",
        [](py::bytes password, py::bytes hashed) {
          std::string p = password, h = hashed;
          py::gil_scoped_release nogil;
          return drtc::bcrypt_checkpw(p, h);
        },
        py::arg("password"), py::arg("hashed"));
  m.def("bcrypt_gensalt",
        [](int cost, py::bytes random16, std::string minor) {
          std::string r = random16;
          if (r.size() != 16) throw std::invalid_argument("need 16 random bytes");
          return py::bytes(drtc::bcrypt_gensalt(cost, (const uint8_t*)r.data(),
                                                minor.empty() ? 'b' : minor[0]));
        },
        py::arg("cost"), py::arg("random16"), py::arg("minor") = "b");

  py::class_<drtc::LogStore>(m, "LogStore")
      .def(py::init<std::string, bool>(), py::arg("path"), py::arg("fsync") = false)
      .def("size", &drtc::LogStore::size)
      .def("append",
           [](drtc::LogStore& s, int64_t term, const std::string& command, py::bytes data) {
             std::string d = data;
             py::gil_scoped_release nogil;
             return s.append(term, command, d);
           })
      .def("get",
           [](drtc::LogStore& s, int64_t index) {
             auto e = s.get(index);
             return py::make_tuple(e.term, e.command, py::bytes(e.data));
           })
      .def("term_at", &drtc::LogStore::term_at)
      .def("truncate_from",
           [](drtc::LogStore& s, int64_t index) {
             py::gil_scoped_release nogil;
             s.truncate_from(index);
           })
      .def("sync", [](drtc::LogStore& s) {
        py::gil_scoped_release nogil;
        s.sync();
      })
      .def("close", &drtc::LogStore::close);

  py::class_<drtc::WordTokenizer>(m, "WordTokenizer")
      .def(py::init<std::vector<std::string>, int32_t, int32_t, std::vector<int32_t>>(),
           py::arg("vocab"), py::arg("byte_base"), py::arg("bos_id"), py::arg("skip_ids"))
      .def_property_readonly("vocab_size", &drtc::WordTokenizer::vocab_size)
      .def("encode",
           [](const drtc::WordTokenizer& t, const std::string& text, bool add_bos) {
             std::vector<int32_t> ids;
             {
               py::gil_scoped_release nogil;
               ids = t.encode(text, add_bos);
             }
             py::list out(ids.size());
             for (size_t i = 0; i < ids.size(); ++i)
               PyList_SET_ITEM(out.ptr(), i, PyLong_FromLong(ids[i]));
             return out;
           },
           py::arg("text"), py::arg("add_bos") = true)
      .def("decode",
           [](const drtc::WordTokenizer& t, const std::vector<int64_t>& ids, bool skip_special) {
             std::string s;
             {
               py::gil_scoped_release nogil;
               s = t.decode(ids, skip_special);
             }
             return py::bytes(s);
           },
           py::arg("ids"), py::arg("skip_special") = true);
}
