// TEST INFRASTRUCTURE: C entry point onto the reference's own MurmurHash64A
// (misc/murmur/MurmurHash2.cpp:99-147), compiled from the reference checkout into
// oracle/_ref/ to pin the oracle's restatement (tests/test_murmur.py).
#include <cstdint>
#include "MurmurHash2.h"

extern "C" uint64_t ref_murmur64a(const void *key, int len, uint64_t seed) {
    return MurmurHash64A(key, len, seed);
}
