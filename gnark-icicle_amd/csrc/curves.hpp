// Curve bundles tying together device field types, host field types and the
// constants each instantiation needs (BN254, BLS12-377; G1 and G2).
#pragma once
#include "curve.hpp"
#include "host_arith.hpp"

namespace gm {

struct CurveBN254 {
  static constexpr int id = 0;
  using Fr = Bn254Fr;
  using Fp = Bn254Fp;
  using G1F = Fe<Bn254Fp>;
  using G2F = Bn254Fp2;
  using HFr = host::HBnFr;
  using HFp = host::HBnFp;
  using HG1F = host::F<host::HBnFp>;
  using HG2F = host::F2<host::HBnFp, -1>;
  static constexpr int FR_BITS = 254;  // r < 2^254
  static constexpr int TWO_ADICITY = 28;
  static constexpr uint64_t COSET_GEN = 5;  // fft FrMultiplicativeGen
};

struct CurveBLS12377 {
  static constexpr int id = 1;
  using Fr = Bls377Fr;
  using Fp = Bls377Fp;
  using G1F = Fe<Bls377Fp>;
  using G2F = Bls377Fp2;
  using HFr = host::HBlsFr;
  using HFp = host::HBlsFp;
  using HG1F = host::F<host::HBlsFp>;
  using HG2F = host::F2<host::HBlsFp, -5>;
  static constexpr int FR_BITS = 253;
  static constexpr int TWO_ADICITY = 47;
  static constexpr uint64_t COSET_GEN = 22;
};

// Select coordinate field by group.
template <class C, bool G2>
struct GroupSel;
template <class C>
struct GroupSel<C, false> {
  using DF = typename C::G1F;
  using HF = typename C::HG1F;
};
template <class C>
struct GroupSel<C, true> {
  using DF = typename C::G2F;
  using HF = typename C::HG2F;
};

}  // namespace gm
