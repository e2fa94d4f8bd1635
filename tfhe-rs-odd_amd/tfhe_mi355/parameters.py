"""Parameter sets of the reference (values copied from the reference's constants; the names are
authoritative -- see SURVEY.md 0.4 for the BASELINE.json annotation mismatch).

  PARAM_MESSAGE_2_CARRY_2_KS_PBS   shortint/parameters/mod.rs:703-717 (alias :1256)
  PARAM_MESSAGE_4_CARRY_4_KS_PBS   shortint/parameters/mod.rs:1063-1077 (alias :1271)
  PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS   shortint/parameters/multi_bit.rs:173-190
  PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS   shortint/parameters/multi_bit.rs:115-132
  MANTICORE_PARAMETERS (fork)      gadget/parameters/mod.rs:224-235
  GADGET_* (fork)                  gadget/parameters/mod.rs:84-222 (DEFAULT, SIMON_40,
                                   ZAMA_TRIVIUM, ASCON_40, SHA3_40, AES_40, AES_23, TFHE_LIB)
  TEST_PARAMS_4_BITS_NATIVE_U64    core_crypto/algorithms/test/mod.rs:56-73
"""
from __future__ import annotations

from dataclasses import dataclass, replace


@dataclass(frozen=True)
class ClassicPBSParameters:
    """Mirror of shortint ClassicPBSParameters (shortint/parameters/mod.rs:60-75)."""

    lwe_dimension: int
    glwe_dimension: int
    polynomial_size: int
    lwe_modular_std_dev: float
    glwe_modular_std_dev: float
    pbs_base_log: int
    pbs_level: int
    ks_base_log: int
    ks_level: int
    message_modulus: int
    carry_modulus: int
    encryption_key_choice: str = "Big"  # "Big" = KS -> PBS order (PBSOrder::KeyswitchBootstrap)
    grouping_factor: int = 0            # > 0: MultiBitPBSParameters
    name: str = ""

    @property
    def big_lwe_dimension(self) -> int:
        return self.glwe_dimension * self.polynomial_size

    @property
    def delta(self) -> int:
        return (1 << 63) // (self.message_modulus * self.carry_modulus)

    def with_(self, **kw) -> "ClassicPBSParameters":
        return replace(self, **kw)


PARAM_MESSAGE_2_CARRY_2_KS_PBS = ClassicPBSParameters(
    lwe_dimension=742, glwe_dimension=1, polynomial_size=2048,
    lwe_modular_std_dev=0.000007069849454709433,
    glwe_modular_std_dev=0.00000000000000029403601535432533,
    pbs_base_log=23, pbs_level=1, ks_base_log=3, ks_level=5,
    message_modulus=4, carry_modulus=4, name="PARAM_MESSAGE_2_CARRY_2_KS_PBS")
PARAM_MESSAGE_2_CARRY_2 = PARAM_MESSAGE_2_CARRY_2_KS_PBS

PARAM_MESSAGE_4_CARRY_4_KS_PBS = ClassicPBSParameters(
    lwe_dimension=996, glwe_dimension=1, polynomial_size=32768,
    lwe_modular_std_dev=0.00000006767666038309478,
    glwe_modular_std_dev=0.0000000000000000002168404344971009,
    pbs_base_log=15, pbs_level=2, ks_base_log=3, ks_level=7,
    message_modulus=16, carry_modulus=16, name="PARAM_MESSAGE_4_CARRY_4_KS_PBS")
PARAM_MESSAGE_4_CARRY_4 = PARAM_MESSAGE_4_CARRY_4_KS_PBS

PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS = ClassicPBSParameters(
    lwe_dimension=888, glwe_dimension=1, polynomial_size=2048,
    lwe_modular_std_dev=0.0000006125031601933181,
    glwe_modular_std_dev=0.0000000000000003152931493498455,
    pbs_base_log=21, pbs_level=1, ks_base_log=7, ks_level=2,
    message_modulus=4, carry_modulus=4, grouping_factor=3,
    name="PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS")

PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS = ClassicPBSParameters(
    lwe_dimension=818, glwe_dimension=1, polynomial_size=2048,
    lwe_modular_std_dev=0.000002226459789930014,
    glwe_modular_std_dev=0.0000000000000003152931493498455,
    pbs_base_log=22, pbs_level=1, ks_base_log=5, ks_level=3,
    message_modulus=4, carry_modulus=4, grouping_factor=2,
    name="PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS")

# fork: GadgetParameters carry no message/carry moduli; 2 x 2 used here for LUT boxes
MANTICORE_PARAMETERS = ClassicPBSParameters(
    lwe_dimension=754, glwe_dimension=1, polynomial_size=1024,
    lwe_modular_std_dev=8.829486224734387e-11,
    glwe_modular_std_dev=5.871712650082723e-15,
    pbs_base_log=15, pbs_level=2, ks_base_log=4, ks_level=3,
    message_modulus=2, carry_modulus=2, name="MANTICORE_PARAMETERS")



def _gadget(name, n, k, N, lwe_std, glwe_std, pbs_bl, pbs_l, ks_bl, ks_l, choice):
    return ClassicPBSParameters(lwe_dimension=n, glwe_dimension=k, polynomial_size=N, lwe_modular_std_dev=lwe_std,
                                glwe_modular_std_dev=glwe_std, pbs_base_log=pbs_bl, pbs_level=pbs_l,
                                ks_base_log=ks_bl, ks_level=ks_l, message_modulus=2, carry_modulus=2,
                                encryption_key_choice=choice, name=name)


# the fork's other GadgetParameters (k = 2, 3, 5 at N = 256..1024)
GADGET_DEFAULT_PARAMETERS = _gadget("GADGET_DEFAULT_PARAMETERS", 722, 2, 512, 0.000013071021089943935,
                                    0.00000004990272175010415, 6, 3, 3, 4, "Small")
GADGET_SIMON_PARAMETERS_40 = _gadget("GADGET_SIMON_PARAMETERS_40", 684, 3, 512, 1.52587890625e-05,
                                     9.313225746154785e-10, 10, 2, 3, 4, "Big")
GADGET_ZAMA_TRIVIUM_PARAMETERS = _gadget("GADGET_ZAMA_TRIVIUM_PARAMETERS", 684, 3, 512, 0.0000204378,
                                         0.000000000000345253, 18, 1, 4, 3, "Small")
GADGET_ASCON_PARAMETERS_40 = _gadget("GADGET_ASCON_PARAMETERS_40", 740, 2, 1024, 1.9073486328125e-06,
                                     9.313225746154785e-10, 7, 3, 5, 3, "Big")
GADGET_SHA3_PARAMETERS_40 = _gadget("GADGET_SHA3_PARAMETERS_40", 676, 5, 256, 0.0009765625,
                                    0.0000000000000000008673617379884035, 14, 1, 4, 3, "Big")
GADGET_AES_PARAMETERS_40 = _gadget("GADGET_AES_PARAMETERS_40", 708, 3, 512, 3.0517578125e-05,
                                   9.313225746154785e-10, 6, 4, 2, 7, "Big")
GADGET_AES_PARAMETERS_23 = _gadget("GADGET_AES_PARAMETERS_23", 672, 3, 512, 0.0000000010797982869590127,
                                   0.0000000000000000008673617379884035, 7, 3, 3, 4, "Big")
GADGET_TFHE_LIB_PARAMETERS = _gadget("GADGET_TFHE_LIB_PARAMETERS", 830, 2, 1024, 0.000001412290588219445,
                                     0.00000000000000029403601535432533, 23, 1, 5, 3, "Small")
GADGET_ALL = [GADGET_DEFAULT_PARAMETERS, GADGET_SIMON_PARAMETERS_40, GADGET_ZAMA_TRIVIUM_PARAMETERS,
              GADGET_ASCON_PARAMETERS_40, GADGET_SHA3_PARAMETERS_40, GADGET_AES_PARAMETERS_40,
              GADGET_AES_PARAMETERS_23, GADGET_TFHE_LIB_PARAMETERS]

TEST_PARAMS_4_BITS_NATIVE_U64 = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(name="TEST_PARAMS_4_BITS_NATIVE_U64")

ALL = {p.name: p for p in [PARAM_MESSAGE_2_CARRY_2_KS_PBS, PARAM_MESSAGE_4_CARRY_4_KS_PBS,
                           PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS,
                           PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS, MANTICORE_PARAMETERS] + GADGET_ALL}
