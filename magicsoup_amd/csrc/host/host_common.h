// Helpers shared by the OpenMP host module (_host).
#pragma once
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstdint>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "ms_common.h"

namespace py = pybind11;

namespace ms_host {

// Process-wide seed sequence for the host RNG streams. Every parallel region derives one
// independent engine per work item from (global seed, call counter, item index), so results depend
// only on the seed and the call order, never on the OpenMP schedule.
uint64_t next_call_seed();
void set_seed(uint64_t seed);

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline std::mt19937_64 item_engine(uint64_t call_seed, uint64_t item) {
  return std::mt19937_64(splitmix64(call_seed ^ splitmix64(item + 0x1234567ull)));
}

// Owning translation tables built from the dictionaries of a Genetics object.
struct HostTables {
  uint8_t is_start[64], is_stop[64], one_codon[64];
  std::vector<uint8_t> dom_type;
  std::vector<uint16_t> two_codon;
  ms::TransTables t{};

  HostTables(const HostTables&) = delete;  // `t` points into this object's own arrays
  HostTables& operator=(const HostTables&) = delete;
  HostTables(const std::vector<std::string>& start_codons, const std::vector<std::string>& stop_codons,
             const std::unordered_map<std::string, int>& domain_map,
             const std::unordered_map<std::string, int>& one_codon_map,
             const std::unordered_map<std::string, int>& two_codon_map, int dom_size, int dom_type_size);
};

int seq_index(const std::string& s);

}  // namespace ms_host
