// pybind11 bindings of the host-side native runtime (module llm_consensus_amd._lib._llmc_rt).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_allocator.h"
#include "gojson.h"
#include "tokenizer.h"

namespace py = pybind11;
using llmc::BlockAllocator;
using llmc::SyntheticTokenizer;

PYBIND11_MODULE(_llmc_rt, m) {
  m.doc() = "llm_consensus_amd native host runtime: tokenizer, paged-KV allocator, Go JSON";

  py::class_<SyntheticTokenizer>(m, "SyntheticTokenizer")
      .def(py::init<int64_t>(), py::arg("vocab_size"))
      .def("encode",
           [](const SyntheticTokenizer& t, py::bytes text) {
             std::string s = text;
             std::vector<int32_t> ids;
             {
               py::gil_scoped_release nogil;
               ids = t.encode(s);
             }
             return ids;
           })
      .def("decode_bytes",
           [](const SyntheticTokenizer& t, const std::vector<int32_t>& ids) {
             return py::bytes(t.decode(ids.data(), static_cast<int64_t>(ids.size())));
           })
      .def("piece_bytes", [](const SyntheticTokenizer& t, int32_t id) { return py::bytes(t.piece(id)); })
      .def_property_readonly("vocab_size", &SyntheticTokenizer::vocab_size)
      .def_property_readonly("bos_id", &SyntheticTokenizer::bos_id)
      .def_property_readonly("eos_id", &SyntheticTokenizer::eos_id)
      .def_property_readonly("num_pieces", &SyntheticTokenizer::num_pieces);

  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int64_t, int64_t>(), py::arg("num_blocks"), py::arg("block_size"))
      .def("allocate", &BlockAllocator::allocate)
      .def("free", &BlockAllocator::free)
      .def("incref", &BlockAllocator::incref)
      .def("refcount", &BlockAllocator::refcount)
      .def("blocks_for", &BlockAllocator::blocks_for)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size);

  m.def("go_json_string",
        [](py::bytes utf8) {
          std::string s = utf8;
          return py::bytes(llmc::go_json_string(s));
        },
        "Encode UTF-8 bytes as a Go encoding/json string literal (HTML-escaped).");
}
