"""Parameter sets of the reference (values copied from the reference's constants; the names are
authoritative -- see SURVEY.md 0.4 for the BASELINE.json annotation mismatch).

  PARAM_MESSAGE_<m>_CARRY_<c>_{KS_PBS,PBS_KS}   shortint/parameters/mod.rs:598-1201 (every set; table below)
  PARAM_MESSAGE_2_CARRY_2_KS_PBS   shortint/parameters/mod.rs:703-717 (alias :1256)
  PARAM_MESSAGE_4_CARRY_4_KS_PBS   shortint/parameters/mod.rs:1063-1077 (alias :1271)
  PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS   shortint/parameters/multi_bit.rs:173-190
  PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS   shortint/parameters/multi_bit.rs:115-132
  PARAM_MULTI_BIT_MESSAGE_{1_CARRY_1,3_CARRY_3}_GROUP_{2,3}_KS_PBS   multi_bit.rs:96-114,134-153,154-172,192-210
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

# the other multi-bit sets (shortint/parameters/multi_bit.rs:96-153, 154-210)
PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_2_KS_PBS = ClassicPBSParameters(
    lwe_dimension=764, glwe_dimension=3, polynomial_size=512,
    lwe_modular_std_dev=0.000006025673585415336, glwe_modular_std_dev=0.0000000000039666089171633006,
    pbs_base_log=18, pbs_level=1, ks_base_log=6, ks_level=2, message_modulus=2, carry_modulus=2,
    grouping_factor=2, name="PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_2_KS_PBS")
PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_2_KS_PBS = ClassicPBSParameters(
    lwe_dimension=922, glwe_dimension=1, polynomial_size=8192,
    lwe_modular_std_dev=0.0000003272369292345697, glwe_modular_std_dev=0.0000000000000000002168404344971009,
    pbs_base_log=14, pbs_level=2, ks_base_log=4, ks_level=4, message_modulus=8, carry_modulus=8,
    grouping_factor=2, name="PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_2_KS_PBS")
PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_3_KS_PBS = ClassicPBSParameters(
    lwe_dimension=765, glwe_dimension=3, polynomial_size=512,
    lwe_modular_std_dev=0.000005915594083804978, glwe_modular_std_dev=0.0000000000039666089171633006,
    pbs_base_log=18, pbs_level=1, ks_base_log=6, ks_level=2, message_modulus=2, carry_modulus=2,
    grouping_factor=3, name="PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_3_KS_PBS")
PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS = ClassicPBSParameters(
    lwe_dimension=972, glwe_dimension=1, polynomial_size=8192,
    lwe_modular_std_dev=0.00000013016688349592805, glwe_modular_std_dev=0.0000000000000000002168404344971009,
    pbs_base_log=14, pbs_level=2, ks_base_log=6, ks_level=3, message_modulus=8, carry_modulus=8,
    grouping_factor=3, name="PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS")
MULTI_BIT_ALL = {p.name: p for p in [
    PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_2_KS_PBS, PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS,
    PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_2_KS_PBS, PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_3_KS_PBS,
    PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS, PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS]}

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

# Every shortint ClassicPBSParameters set of the reference (shortint/parameters/mod.rs:598-1201):
# (name, source line, n, k, N, lwe std, glwe std, pbs base_log, pbs level, ks base_log, ks level,
#  message modulus, carry modulus, encryption key choice)
_SHORTINT_TABLE = [
    ("PARAM_MESSAGE_1_CARRY_0_KS_PBS", 598, 678, 5, 256, 0.000022810107419132102, 0.00000000037411618952047216,
     15, 1, 5, 2, 2, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_1_KS_PBS", 613, 684, 3, 512, 0.00002043784477291318, 0.0000000000034525330484572114,
     18, 1, 4, 3, 2, 2, "Big"),
    ("PARAM_MESSAGE_2_CARRY_0_KS_PBS", 628, 656, 2, 512, 0.000034119201269311964, 0.00000004053919869756513,
     8, 2, 3, 4, 4, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_2_KS_PBS", 643, 742, 2, 1024, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 4, 3, 2, 4, "Big"),
    ("PARAM_MESSAGE_2_CARRY_1_KS_PBS", 658, 742, 2, 1024, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 4, 3, 4, 2, "Big"),
    ("PARAM_MESSAGE_3_CARRY_0_KS_PBS", 673, 742, 2, 1024, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 4, 3, 8, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_3_KS_PBS", 688, 745, 1, 2048, 0.000006692125069956277, 0.00000000000000029403601535432533,
     23, 1, 3, 5, 2, 8, "Big"),
    ("PARAM_MESSAGE_2_CARRY_2_KS_PBS", 703, 742, 1, 2048, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 3, 5, 4, 4, "Big"),
    ("PARAM_MESSAGE_3_CARRY_1_KS_PBS", 718, 742, 1, 2048, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 3, 5, 8, 2, "Big"),
    ("PARAM_MESSAGE_4_CARRY_0_KS_PBS", 733, 742, 1, 2048, 0.000007069849454709433, 0.00000000000000029403601535432533,
     23, 1, 3, 5, 16, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_4_KS_PBS", 748, 807, 1, 4096, 0.0000021515145918907506, 0.0000000000000000002168404344971009,
     15, 2, 3, 5, 2, 16, "Big"),
    ("PARAM_MESSAGE_2_CARRY_3_KS_PBS", 763, 856, 1, 4096, 0.0000008775214009854235, 0.0000000000000000002168404344971009,
     22, 1, 3, 6, 4, 8, "Big"),
    ("PARAM_MESSAGE_3_CARRY_2_KS_PBS", 778, 812, 1, 4096, 0.0000019633637461248447, 0.0000000000000000002168404344971009,
     22, 1, 3, 5, 8, 4, "Big"),
    ("PARAM_MESSAGE_4_CARRY_1_KS_PBS", 793, 808, 1, 4096, 0.0000021124945159091033, 0.0000000000000000002168404344971009,
     22, 1, 3, 5, 16, 2, "Big"),
    ("PARAM_MESSAGE_5_CARRY_0_KS_PBS", 808, 807, 1, 4096, 0.0000021515145918907506, 0.0000000000000000002168404344971009,
     22, 1, 3, 5, 32, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_5_KS_PBS", 823, 864, 1, 8192, 0.000000757998020150446, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 2, 32, "Big"),
    ("PARAM_MESSAGE_2_CARRY_4_KS_PBS", 838, 864, 1, 8192, 0.000000757998020150446, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 4, 16, "Big"),
    ("PARAM_MESSAGE_3_CARRY_3_KS_PBS", 853, 864, 1, 8192, 0.000000757998020150446, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 8, 8, "Big"),
    ("PARAM_MESSAGE_4_CARRY_2_KS_PBS", 868, 864, 1, 8192, 0.000000757998020150446, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 16, 4, "Big"),
    ("PARAM_MESSAGE_5_CARRY_1_KS_PBS", 883, 875, 1, 8192, 0.0000006197725091905067, 0.0000000000000000002168404344971009,
     22, 1, 3, 6, 32, 2, "Big"),
    ("PARAM_MESSAGE_6_CARRY_0_KS_PBS", 898, 915, 1, 8192, 0.00000029804653749339636, 0.0000000000000000002168404344971009,
     22, 1, 4, 4, 64, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_6_KS_PBS", 913, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     11, 3, 3, 6, 2, 64, "Big"),
    ("PARAM_MESSAGE_2_CARRY_5_KS_PBS", 928, 934, 1, 16384, 0.00000021050318566634375, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 4, 32, "Big"),
    ("PARAM_MESSAGE_3_CARRY_4_KS_PBS", 943, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 8, 16, "Big"),
    ("PARAM_MESSAGE_4_CARRY_3_KS_PBS", 958, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 16, 8, "Big"),
    ("PARAM_MESSAGE_5_CARRY_2_KS_PBS", 973, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 32, 4, "Big"),
    ("PARAM_MESSAGE_6_CARRY_1_KS_PBS", 988, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 64, 2, "Big"),
    ("PARAM_MESSAGE_7_CARRY_0_KS_PBS", 1003, 930, 1, 16384, 0.00000022649232786295453, 0.0000000000000000002168404344971009,
     15, 2, 3, 6, 128, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_7_KS_PBS", 1018, 1004, 1, 32768, 0.00000005845871624688967, 0.0000000000000000002168404344971009,
     11, 3, 3, 7, 2, 128, "Big"),
    ("PARAM_MESSAGE_2_CARRY_6_KS_PBS", 1033, 987, 1, 32768, 0.00000007979529246348835, 0.0000000000000000002168404344971009,
     11, 3, 3, 7, 4, 64, "Big"),
    ("PARAM_MESSAGE_3_CARRY_5_KS_PBS", 1048, 985, 1, 32768, 0.00000008277032914509569, 0.0000000000000000002168404344971009,
     11, 3, 3, 7, 8, 32, "Big"),
    ("PARAM_MESSAGE_4_CARRY_4_KS_PBS", 1063, 996, 1, 32768, 0.00000006767666038309478, 0.0000000000000000002168404344971009,
     15, 2, 3, 7, 16, 16, "Big"),
    ("PARAM_MESSAGE_5_CARRY_3_KS_PBS", 1078, 1020, 1, 32768, 0.000000043618425315728666, 0.0000000000000000002168404344971009,
     15, 2, 4, 5, 32, 8, "Big"),
    ("PARAM_MESSAGE_6_CARRY_2_KS_PBS", 1093, 1018, 1, 32768, 0.000000045244666805696514, 0.0000000000000000002168404344971009,
     15, 2, 4, 5, 64, 4, "Big"),
    ("PARAM_MESSAGE_7_CARRY_1_KS_PBS", 1108, 1017, 1, 32768, 0.0000000460803851108693, 0.0000000000000000002168404344971009,
     15, 2, 4, 5, 128, 2, "Big"),
    ("PARAM_MESSAGE_8_CARRY_0_KS_PBS", 1123, 1017, 1, 32768, 0.0000000460803851108693, 0.0000000000000000002168404344971009,
     15, 2, 4, 5, 256, 1, "Big"),
    ("PARAM_MESSAGE_1_CARRY_1_PBS_KS", 1139, 783, 3, 512, 0.0000033382067621812462, 0.0000000000034525330484572114,
     18, 1, 5, 3, 2, 2, "Small"),
    ("PARAM_MESSAGE_2_CARRY_2_PBS_KS", 1155, 870, 1, 2048, 0.0000006791658447437413, 0.00000000000000029403601535432533,
     23, 1, 4, 4, 4, 4, "Small"),
    ("PARAM_MESSAGE_3_CARRY_3_PBS_KS", 1171, 1025, 1, 8192, 0.00000003980397588319241, 0.0000000000000000002168404344971009,
     15, 2, 4, 5, 8, 8, "Small"),
    ("PARAM_MESSAGE_4_CARRY_4_PBS_KS", 1187, 1214, 1, 32768, 0.0000000012520482863081104, 0.0000000000000000002168404344971009,
     15, 2, 4, 6, 16, 16, "Small"),
]

SHORTINT_ALL = {
    t[0]: ClassicPBSParameters(lwe_dimension=t[2], glwe_dimension=t[3], polynomial_size=t[4], lwe_modular_std_dev=t[5],
                               glwe_modular_std_dev=t[6], pbs_base_log=t[7], pbs_level=t[8], ks_base_log=t[9],
                               ks_level=t[10], message_modulus=t[11], carry_modulus=t[12], encryption_key_choice=t[13],
                               name=t[0])
    for t in _SHORTINT_TABLE}
SHORTINT_SOURCE_LINE = {t[0]: t[1] for t in _SHORTINT_TABLE}
assert SHORTINT_ALL["PARAM_MESSAGE_2_CARRY_2_KS_PBS"] == PARAM_MESSAGE_2_CARRY_2_KS_PBS
assert SHORTINT_ALL["PARAM_MESSAGE_4_CARRY_4_KS_PBS"] == PARAM_MESSAGE_4_CARRY_4_KS_PBS
globals().update(SHORTINT_ALL)

ALL = {p.name: p for p in [PARAM_MESSAGE_2_CARRY_2_KS_PBS, PARAM_MESSAGE_4_CARRY_4_KS_PBS,
                           PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS,
                           PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS, MANTICORE_PARAMETERS] + GADGET_ALL}
ALL.update(SHORTINT_ALL)
ALL.update(MULTI_BIT_ALL)
