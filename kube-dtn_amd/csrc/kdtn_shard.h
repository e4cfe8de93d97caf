// kdtn_shard.h — topology owner shard: hash64(namespace ‖ "/" ‖ name) mod G.
// One definition shared by the exported kdtn_topology_shard (kdtn_intern.cpp) and the
// synthetic generator, so a controller, the generator and the tests place every Topology on
// the same GPU. The key is the informer's object key (cache.MetaNamespaceKeyFunc:
// "namespace/name"), the same string getPod looks peers up by (daemon/kubedtn/handler.go:27-41).
#pragma once
#include <stdint.h>

// callable from host code and, in HIP translation units, from kernels (the sharded ingest
// picks a rank's Topologies on the GPU with the same function)
#if defined(__HIPCC__)
#define KDTN_SHARD_FN __host__ __device__ inline
#else
#define KDTN_SHARD_FN inline
#endif

namespace kdtn {

// FNV-1a 64 over the key bytes, then the murmur3 fmix64 finalizer (FNV's low bits alone are
// weak for short, similar keys like "default/p123").
KDTN_SHARD_FN uint64_t topology_key_hash(const uint8_t* ns, uint32_t ns_len, const uint8_t* name, uint32_t name_len) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < ns_len; ++i) h = (h ^ ns[i]) * 1099511628211ull;
    h = (h ^ (uint8_t)'/') * 1099511628211ull;
    for (uint32_t i = 0; i < name_len; ++i) h = (h ^ name[i]) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}

KDTN_SHARD_FN uint32_t topology_shard(const uint8_t* ns, uint32_t ns_len, const uint8_t* name, uint32_t name_len,
                               uint32_t nshards) {
    return nshards <= 1 ? 0u : (uint32_t)(topology_key_hash(ns, ns_len, name, name_len) % nshards);
}

}  // namespace kdtn
