// Host-side (CPU) native runtime for ytk-learn-amd.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace ytk_native {

int64_t murmur3_128_aslong(const char* data, size_t len, uint32_t seed);

}  // namespace ytk_native
