// kdtn_intern.cpp — host string interning for the C-ABI (kdtn_interner_*).
// Produces deduplicated dictionaries (id equality ⇔ byte equality) with id 0 = "",
// the precondition every kdtn_strtab in include/kdtn.h relies on. Ids are assigned in
// first-seen order, so strings that occur once per link get ids in link order and the
// device-side gathers over per-string tables stay nearly sequential.
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/kdtn.h"
#include "kdtn_shard.h"

namespace {
uint64_t fnv(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h ^ (h >> 29);
}
}  // namespace

struct kdtn_interner {
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> offs{0};
    std::vector<uint32_t> slots;   // id + 1, 0 = empty
    std::vector<uint64_t> hashes;  // per id

    uint32_t size() const { return (uint32_t)(offs.size() - 1); }

    void rehash(size_t cap) {
        slots.assign(cap, 0);
        for (uint32_t id = 0; id < size(); ++id) {
            size_t h = hashes[id] & (cap - 1);
            while (slots[h]) h = (h + 1) & (cap - 1);
            slots[h] = id + 1;
        }
    }

    uint32_t intern(const uint8_t* s, uint32_t n) {
        if ((size() + 1) * 2 > slots.size()) rehash(slots.empty() ? 1024 : slots.size() * 2);
        const uint64_t h = fnv(s, n);
        size_t pos = h & (slots.size() - 1);
        for (;;) {
            const uint32_t v = slots[pos];
            if (!v) break;
            const uint32_t id = v - 1;
            if (hashes[id] == h && offs[id + 1] - offs[id] == n &&
                (n == 0 || std::memcmp(bytes.data() + offs[id], s, n) == 0))
                return id;
            pos = (pos + 1) & (slots.size() - 1);
        }
        const uint32_t id = size();
        bytes.insert(bytes.end(), s, s + n);
        offs.push_back((uint32_t)bytes.size());
        hashes.push_back(h);
        slots[pos] = id + 1;
        return id;
    }
};

extern "C" {

int kdtn_interner_new(kdtn_interner** out) {
    if (!out) return KDTN_EINVAL;
    kdtn_interner* it = new (std::nothrow) kdtn_interner();
    if (!it) return KDTN_ENOMEM;
    it->intern(reinterpret_cast<const uint8_t*>(""), 0);   // id 0 = ""
    *out = it;
    return KDTN_OK;
}

void kdtn_interner_free(kdtn_interner* it) { delete it; }

uint32_t kdtn_intern(kdtn_interner* it, const char* s, uint32_t len) {
    return it->intern(reinterpret_cast<const uint8_t*>(s), len);
}

int kdtn_intern_batch(kdtn_interner* it, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                      uint32_t* ids_out) {
    if (!it || (n && (!offs || !ids_out))) return KDTN_EINVAL;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t a = offs[i], b = offs[i + 1];
        if (b < a || b - a > 0xFFFFFFFFull) return KDTN_EINVAL;
        ids_out[i] = it->intern(bytes + a, (uint32_t)(b - a));
    }
    return KDTN_OK;
}

int kdtn_interner_table(const kdtn_interner* it, kdtn_strtab* out) {
    if (!it || !out) return KDTN_EINVAL;
    out->bytes = it->bytes.data();
    out->offs = it->offs.data();
    out->n = it->size();
    return KDTN_OK;
}

}  // extern "C"

extern "C" uint32_t kdtn_topology_shard(const uint8_t* ns, uint32_t ns_len, const uint8_t* name,
                                        uint32_t name_len, uint32_t nshards) {
    return kdtn::topology_shard(ns, ns_len, name, name_len, nshards);
}
