// wire.hpp — host side of the state-message wire format (System.Text.Json).
//
// PNCounterMsg payloads are decoded on the GPU (csrc/json.hip); this header holds what the host needs
// around that: the PNCounterMsg writer (PNCounters.cs:46-49, the producer of those payloads:
// GetLastSynchronizedUpdate().Encode() in SafeCRDT.Update, BFT-CRDT/SafeCRDTs/SafeCRDT.cs:49) and the
// ORSetMsg<string> reader/writer (ORSet.cs:56-69), whose element strings are interned on the host.
// The accepted decode contract is the one stated in oracle/json.hpp (the checker's restatement).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "janus_host.hpp"

namespace janus::wire {

// Guid.ToString("D") (lower-case) of C# Guid bytes lo = b0..b7, hi = b8..b15; appends 36 chars.
void AppendGuidD(std::string& out, const Guid& g);
bool ParseGuidD(std::string_view s, Guid& g);

// PNCounterMsg.Encode of a state whose pVector and nVector both list the k replicas g[0..k) in that
// order with values p[i] / n[i]: {"pVector":{"<g>":p,...},"nVector":{"<g>":n,...}}.  Appends.
void AppendPNCounterMsg(std::string& out, const Guid* g, const int64_t* p, const int64_t* n, size_t k);

// ORSetMsg<string?> codec.  Decode throws EngineError(JG_EINVAL) where System.Text.Json rejects the payload or
// the reference's Merge would throw (oracle/json.hpp's contract: unknown members skipped, repeats last-wins).
std::string EncodeORSetMsg(const ORSetState& m);
ORSetState DecodeORSetMsg(std::string_view bytes);

// The decoded state in ORSet.Merge's walk: fn(ctx, side, name, is_null, tags, n) once per entry — side 0 =
// addSet / nullAddGuid, 1 = removeSet / nullRemoveGuid; is_null = the null tag set (name empty, reported last,
// after every element: ORSet.cs:255-282).  `name` and `tags` are valid during the call.  Accepts and rejects
// exactly what DecodeORSetMsg does (nothing is reported for a rejected payload).
using ORSetEntryFn = void (*)(void* ctx, int side, std::string_view name, bool is_null, const Guid* tags, size_t n);
void ScanORSetMsg(std::string_view bytes, ORSetEntryFn fn, void* ctx);

}  // namespace janus::wire
