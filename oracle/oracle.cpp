// oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
// Safe-CRDT wrapper and SafeCRDTManager restatement: BFT-CRDT/SafeCRDTs/SafeCRDT.cs:19-83 and
// BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:61-198.
#include "oracle.hpp"

#include "json.hpp"

namespace oracle {

SafeCRDT::SafeCRDT(Guid uid, std::string k, CrdtType t, GuidGen& g, SafeCRDTManager* m)
    : guid(uid), key(std::move(k)), type(t), gen(&g), sm(m) {
    // SafeCRDTManager.cs:64-69: the prospective instance comes from RM, the stable one is a fresh
    // instance of the same type (its own replica Guid, never incremented).
    if (t == CrdtType::PNCounter) { pncProspective.emplace(g); pncStable.emplace(g); }
    else { orProspective.emplace(); orStable.emplace(); }
}

StateMsg SafeCRDT::ProspectiveState() const {
    StateMsg m; m.type = type;
    if (type == CrdtType::PNCounter) m.pnc = pncProspective->pnc.GetLastSynchronizedUpdate();
    else m.orset = orProspective->orset.GetLastSynchronizedUpdate();
    return m;
}

// SafeCRDT.cs:39-62 — apply to the prospective copy, snapshot the full state into a
// NetworkProtocol{uid, CRDTMsg, state}, track it when safe, hand it to the batcher.
Result SafeCRDT::Update(int op, const std::vector<Arg>& args, bool isSafe, uint64_t origin) {
    NetworkProtocol syncMsg;
    Result r;
    if (type == CrdtType::PNCounter) r = pncProspective->Update(op, args);
    else r = orProspective->Update(op, args, *gen);
    syncMsg.uid = guid;
    syncMsg.syncMsgType = NetworkProtocol::CRDTMsg;
    syncMsg.message = ProspectiveState();
    syncMsg.bytes = type == CrdtType::PNCounter ? json::EncodePNC(syncMsg.message.pnc) : json::EncodeORSet(syncMsg.message.orset);
    syncMsg.seq = sm->nextSeq++;
    if (isSafe && origin != 0) sm->safeUpdateTracker.emplace(syncMsg.seq, origin);
    sm->ActualPropagateSyncMsg(syncMsg, sm->clock_ms);
    return r;
}

Result SafeCRDT::QueryStable(const std::vector<Arg>& args) const {
    return type == CrdtType::PNCounter ? pncStable->Query() : orStable->Query(args);
}
Result SafeCRDT::QueryProspective(const std::vector<Arg>& args) const {
    return type == CrdtType::PNCounter ? pncProspective->Query() : orProspective->Query(args);
}

// SafeCRDT.cs:80-83 — decode + ApplySynchronizedUpdate on the stable copy.  Encoded messages are
// decoded with the stable copy's own codec (json::JsonException where Decode throws); a decoded
// message of the other CRDT type is ORSet.cs:288-291's NotSupportedException (PNCounter casts:
// InvalidCast).
void SafeCRDT::ApplyUpdateStable(const NetworkProtocol& msg) {
    if (!msg.bytes.empty()) {
        if (type == CrdtType::PNCounter) pncStable->pnc.ApplySynchronizedUpdate(json::DecodePNC<int32_t>(msg.bytes));
        else orStable->orset.ApplySynchronizedUpdate(json::DecodeORSet(msg.bytes));
        return;
    }
    if (msg.message.type != type) {
        if (type == CrdtType::ORSet) throw NotSupportedException("ReceivedUpdate does not support type");
        throw InvalidCastException("Specified cast is not valid.");
    }
    if (type == CrdtType::PNCounter) pncStable->pnc.ApplySynchronizedUpdate(msg.message.pnc);
    else orStable->orset.ApplySynchronizedUpdate(msg.message.orset);
}

SafeCRDT& SafeCRDTManager::CreateSafeCRDT(const std::string& key, CrdtType t) {
    return CreateSafeCRDT(key, t, gen.next());
}

SafeCRDT& SafeCRDTManager::CreateSafeCRDT(const std::string& key, CrdtType t, const Guid& uid) {
    auto sc = std::make_unique<SafeCRDT>(uid, key, t, gen, this);
    SafeCRDT* raw = sc.get();
    safeCRDTs[key] = raw;
    safeCRDTsIndexedByuid[uid] = std::move(sc);
    return *raw;
}

void SafeCRDTManager::HandleAfterConsensusUpdates(const std::vector<std::vector<UpdateMessage>>& updates) {
    for (const auto& list : updates)
        for (const auto& block : list)
            for (const auto& u : block.update) {
                if (u.syncMsgType == NetworkProtocol::ManagerMsg_Create || u.uid.is_empty()) continue;  // :133-134
                auto it = safeCRDTsIndexedByuid.find(u.uid);                                            // :136
                if (it == safeCRDTsIndexedByuid.end()) continue;
                it->second->ApplyUpdateStable(u);                                                        // :139
                auto tr = safeUpdateTracker.find(u.seq);                                                 // :141-142
                if (tr != safeUpdateTracker.end()) { notified.push_back(tr->second); safeUpdateTracker.erase(tr); }
            }
}

void SafeCRDTManager::ActualPropagateSyncMsg(const NetworkProtocol& msg, double now_ms) {
    clientUpdateBuffer.push_back(msg);
    if ((int)clientUpdateBuffer.size() >= clientBatchSize || (now_ms - lastSubmittedMs) > 100.0) {
        OrderedDict<Guid, NetworkProtocol, GuidHash> appearedObjects;
        std::vector<NetworkProtocol> msgs;
        while (!clientUpdateBuffer.empty()) {
            NetworkProtocol np = clientUpdateBuffer.front();  // TryDequeue happens first ...
            clientUpdateBuffer.pop_front();
            if (!((int)msgs.size() < clientBatchSize)) break;  // ... so this message is dropped (:175)
            if (!safeUpdateTracker.count(np.seq)) appearedObjects[np.uid] = np;
            else msgs.push_back(np);
        }
        for (const auto& kv : appearedObjects) msgs.push_back(kv.second);
        if (!msgs.empty()) {
            submitted.push_back(UpdateMessage{msgs});
            lastSubmittedMs = now_ms;
        }
    }
}

}  // namespace oracle
