// pybind.cpp -- Python module _rsmi_host: the C++ host layer (infectious.hpp,
// shard_plugin.hpp) for the tests and bench, so they drive the same C++ code
// a native caller would.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "infectious.hpp"
#include "plugin_latency.hpp"
#include "shard_plugin.hpp"

namespace py = pybind11;
using namespace rsmi_host;

namespace {

std::vector<uint8_t> to_vec(const py::bytes& b) {
    const std::string s = b;
    return std::vector<uint8_t>(s.begin(), s.end());
}
py::bytes to_bytes(const std::vector<uint8_t>& v) {
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

struct StatusError : std::runtime_error {
    int code;
    StatusError(const Status& s) : std::runtime_error(s.msg), code(s.code) {}
};

void check(const Status& s) {
    if (!s.ok()) throw StatusError(s);
}

}  // namespace

PYBIND11_MODULE(_rsmi_host, m) {
    m.doc() = "C++ host layer of the MI355X RS engine (ShardPlugin mirror, Shard codec)";
    static py::exception<StatusError> exc(m, "HostError");
    py::register_exception_translator([](std::exception_ptr p) {
        try {
            if (p) std::rethrow_exception(p);
        } catch (const StatusError& e) {
            PyErr_SetObject(exc.ptr(), py::make_tuple(e.what(), e.code).ptr());
        }
    });

    py::class_<Share>(m, "Share")
        .def(py::init([](int n, const py::bytes& d) { return Share{n, to_vec(d)}; }))
        .def_readwrite("Number", &Share::Number)
        .def_property("Data", [](const Share& s) { return to_bytes(s.Data); },
                      [](Share& s, const py::bytes& b) { s.Data = to_vec(b); })
        .def("DeepCopy", &Share::DeepCopy);

    py::class_<FEC, std::shared_ptr<FEC>>(m, "FEC")
        .def("Required", &FEC::Required)
        .def("Total", &FEC::Total)
        .def("Encode",
             [](FEC& f, const py::bytes& input, const std::function<void(Share)>& output) {
                 const std::string s = input;
                 check(f.Encode(reinterpret_cast<const uint8_t*>(s.data()), s.size(),
                                [&](const ShareView& v) { output(v.DeepCopy()); }));
             })
        .def("EncodeBatch",
             [](FEC& f, const std::vector<py::bytes>& inputs) {
                 // equal-length messages (rs_encode_batch); None where a message failed
                 std::vector<std::string> keep(inputs.begin(), inputs.end());
                 std::vector<const uint8_t*> ptrs;
                 for (const std::string& x : keep) ptrs.push_back(reinterpret_cast<const uint8_t*>(x.data()));
                 const size_t len = keep.empty() ? 0 : keep[0].size();
                 for (const std::string& x : keep)
                     if (x.size() != len) throw std::invalid_argument("EncodeBatch: messages of unequal length");
                 std::vector<std::vector<uint8_t>> par;
                 std::vector<Status> st;
                 {
                     py::gil_scoped_release nogil;
                     f.EncodeBatch(ptrs, len, &par, &st);
                 }
                 py::list res;
                 for (size_t b = 0; b < par.size(); ++b)
                     res.append(st[b].ok() ? py::object(to_bytes(par[b])) : py::object(py::none()));
                 return res;
             })
        .def("DecodeBatch",
             [](FEC& f, std::vector<std::vector<Share>> msgs) {
                 std::vector<std::vector<uint8_t>> outs;
                 std::vector<Status> st;
                 f.DecodeBatch(msgs, &outs, &st);
                 py::list res;
                 for (size_t b = 0; b < outs.size(); ++b)
                     res.append(st[b].ok() ? py::object(to_bytes(outs[b])) : py::object(py::none()));
                 return res;
             })
        .def("Decode", [](FEC& f, py::object /*dst*/, std::vector<Share>& shares) {
            std::vector<uint8_t> out;
            check(f.Decode(&out, shares));
            return py::make_tuple(to_bytes(out), shares);
        });

    m.def("NewFEC", [](int k, int n) {
        std::shared_ptr<FEC> f;
        check(NewFEC(k, n, &f));
        return f;
    });

    py::class_<Shard>(m, "Shard")
        .def(py::init<>())
        .def(py::init([](const py::bytes& sig, const py::bytes& data, uint64_t num, uint64_t total,
                         uint64_t need) {
                 Shard s;
                 s.FileSignature = to_vec(sig);
                 s.ShardData = to_vec(data);
                 s.ShardNumber = num;
                 s.TotalShards = total;
                 s.MinimumNeededShards = need;
                 return s;
             }),
             py::arg("FileSignature") = py::bytes(), py::arg("ShardData") = py::bytes(),
             py::arg("ShardNumber") = 0, py::arg("TotalShards") = 0,
             py::arg("MinimumNeededShards") = 0)
        .def_property("FileSignature", [](const Shard& s) { return to_bytes(s.FileSignature); },
                      [](Shard& s, const py::bytes& b) { s.FileSignature = to_vec(b); })
        .def_property("ShardData", [](const Shard& s) { return to_bytes(s.ShardData); },
                      [](Shard& s, const py::bytes& b) { s.ShardData = to_vec(b); })
        .def_readwrite("ShardNumber", &Shard::ShardNumber)
        .def_readwrite("TotalShards", &Shard::TotalShards)
        .def_readwrite("MinimumNeededShards", &Shard::MinimumNeededShards)
        .def("Size", &Shard::Size)
        .def("Marshal", [](const Shard& s) { return to_bytes(s.Marshal()); })
        .def("Unmarshal",
             [](Shard& s, const py::bytes& b) {
                 const std::string d = b;
                 check(s.Unmarshal(reinterpret_cast<const uint8_t*>(d.data()), d.size()));
             })
        .def("__eq__", &Shard::operator==);

    py::class_<PeerID>(m, "PeerID")
        .def(py::init([](const std::string& addr, const py::bytes& id) { return PeerID{addr, to_vec(id)}; }))
        .def_readwrite("Address", &PeerID::Address);

    py::class_<ReceiveEvent>(m, "ReceiveEvent")
        .def_readonly("pooled", &ReceiveEvent::pooled)
        .def_readonly("decoded", &ReceiveEvent::decoded)
        .def_readonly("verified", &ReceiveEvent::verified)
        .def_property_readonly("decode_code", [](const ReceiveEvent& e) { return e.decode_status.code; })
        .def_property_readonly("message", [](const ReceiveEvent& e) { return to_bytes(e.message); });

    py::class_<ShardPlugin>(m, "ShardPlugin")
        .def_readwrite("MinimumNeededShards", &ShardPlugin::MinimumNeededShards)
        .def_readwrite("TotalShards", &ShardPlugin::TotalShards)
        .def("Receive",
             [](ShardPlugin& p, const PeerID& sender, const Shard& msg) {
                 // noise calls Receive once per peer connection, concurrently
                 // (main.go:49-52): the GIL is released so Python threads do
                 // too (the sign/verify callbacks take it back).
                 ReceiveEvent ev;
                 Status st;
                 {
                     py::gil_scoped_release nogil;
                     st = p.Receive(sender, msg, &ev);
                 }
                 check(st);
                 return ev;
             })
        .def("ReceiveBatch",
             [](ShardPlugin& p, const std::vector<std::pair<PeerID, Shard>>& msgs) {
                 std::vector<ReceiveEvent> evs;
                 std::vector<Status> sts;
                 {
                     py::gil_scoped_release nogil;
                     p.ReceiveBatch(msgs, &evs, &sts);
                 }
                 std::vector<int> codes;
                 for (const Status& s : sts) codes.push_back(s.code);
                 return py::make_tuple(evs, codes);
             })
        .def("prepareShards",
             [](ShardPlugin& p, const PeerID& self, py::object input) {
                 std::vector<Shard> out;
                 if (input.is_none()) {
                     check(p.prepareShards(self, nullptr, &out));
                 } else {
                     const std::vector<uint8_t> v = to_vec(input.cast<py::bytes>());
                     check(p.prepareShards(self, &v, &out));
                 }
                 return out;
             })
        .def("prepareShardsBatch",
             [](ShardPlugin& p, const PeerID& self, const std::vector<py::bytes>& inputs) {
                 std::vector<std::vector<uint8_t>> in;
                 for (const py::bytes& b : inputs) in.push_back(to_vec(b));
                 std::vector<std::vector<Shard>> out;
                 std::vector<Status> sts;
                 {
                     py::gil_scoped_release nogil;
                     p.prepareShardsBatch(self, in, &out, &sts);
                 }
                 std::vector<int> codes;
                 for (const Status& s : sts) codes.push_back(s.code);
                 return py::make_tuple(out, codes);
             })
        .def("HashBytes",
             [](const ShardPlugin& p, const std::vector<py::bytes>& msgs) {
                 std::vector<std::vector<uint8_t>> in, out;
                 for (const py::bytes& b : msgs) in.push_back(to_vec(b));
                 check(p.HashBytes(in, &out));
                 py::list res;
                 for (const auto& d : out) res.append(to_bytes(d));
                 return res;
             })
        .def_readwrite("HashLen", &ShardPlugin::HashLen)
        .def("ShardAndBroadcast",
             [](ShardPlugin& p, const PeerID& self, const py::bytes& input,
                const std::function<void(Shard)>& broadcast) {
                 const std::vector<uint8_t> v = to_vec(input);
                 check(p.ShardAndBroadcast(self, &v, [&](const Shard& s) { broadcast(s); }));
             })
        .def("ShardAndBroadcastWire",
             [](ShardPlugin& p, const PeerID& self, py::object input, const std::function<void(py::bytes)>& broadcast) {
                 if (input.is_none()) {
                     check(p.ShardAndBroadcastWire(self, nullptr, [](const uint8_t*, size_t) {}));
                     return;
                 }
                 const std::vector<uint8_t> v = to_vec(input.cast<py::bytes>());
                 check(p.ShardAndBroadcastWire(self, &v, [&](const uint8_t* w, size_t len) {
                     broadcast(py::bytes(reinterpret_cast<const char*>(w), len));
                 }));
             })
        .def("ReceiveMove",
             [](ShardPlugin& p, const PeerID& sender, Shard msg) {
                 // Receive(Shard&&): the pooled share keeps the message's bytes
                 ReceiveEvent ev;
                 Status st;
                 {
                     py::gil_scoped_release nogil;
                     st = p.Receive(sender, std::move(msg), &ev);
                 }
                 check(st);
                 return ev;
             })
        .def("shardInput",
             [](ShardPlugin& p, const py::bytes& input) {
                 std::vector<Share> out;
                 check(p.shardInput(to_vec(input), &out));
                 return out;
             })
        .def("PoolSize", [](const ShardPlugin& p, const py::bytes& sig) { return p.PoolSize(to_vec(sig)); });

    m.def("NewShardPlugin",
          [](std::function<py::bytes(py::bytes)> sign, std::function<bool(py::bytes, py::bytes)> verify,
             int k, int n, int hash_len) {
              // None -> no signing / no verification (the callbacks stay empty)
              Signer s;
              Verifier v;
              if (sign)
                  s = [sign](const std::vector<uint8_t>& msg) {
                      py::gil_scoped_acquire g;
                      return to_vec(sign(to_bytes(msg)));
                  };
              if (verify)
                  v = [verify](const std::vector<uint8_t>& msg, const std::vector<uint8_t>& sig) {
                      py::gil_scoped_acquire g;
                      return verify(to_bytes(msg), to_bytes(sig));
                  };
              return NewShardPlugin(s, v, k, n, hash_len).release();
          },
          py::arg("sign"), py::arg("verify"), py::arg("k"), py::arg("n"), py::arg("hash_len") = 0,
          py::return_value_policy::take_ownership);
    m.def("serializeMessage", [](const PeerID& id, const py::bytes& msg) {
        return to_bytes(serializeMessage(id, to_vec(msg)));
    });
    m.def("plugin_latency",
          [](const py::bytes& blob, int k, int n, const std::vector<int>& dropped, int reps) {
              const std::vector<uint8_t> b = to_vec(blob);
              std::map<std::string, double> out;
              Status st;
              {
                  py::gil_scoped_release nogil;
                  st = PluginLatency(b, k, n, dropped, reps, &out);
              }
              check(st);
              return out;
          },
          "The config-1 plugin path timed in C++ (plugin_latency.cpp): median ms per step.");
    m.def("largestPrimeFactors", &largestPrimeFactors);
    m.def("StatusText", &StatusText);
}
