"""Kernel alternates the shipped libozec.so holds (ozone_amd/csrc/kernels.hpp kGfVariants / kCrcVariants), by kernel
family.  The GPU parity tests parametrize over these lists, and tests/test_variants.py (CPU) checks that their union is
exactly what the library reports (ozec_tuning_variants), so no selectable variant goes without a parity test."""

GF = [1, 5, 11]                        # coding kernel gf_code_vec (kernels.hip launch_kr)
CRC_STREAM = [20, 22, 24, 28, 29]                  # streaming CRC kernel (kernels.hip launch_crc_windows)
XOR_FUSED = [2, 3, 4, 5, 20, 21]       # fused XOR codec (kernels.hip launch_enc_crc_kr, R = 1 all-ones)
RS_FUSED = [49, 56, 59, 62, 87, 150, 163, 167, 170, 171, 172, 173, 174, 176, 177,
            187, 189, 190, 191, 192, 193, 194, 196, 220, 221, 222, 231, 234]  # fused RS (launch_encode_crc)
NB_PERSISTENT = [150, 163, 167, 170, 171, 172, 176, 177, 187, 189, 190, 191, 192, 193, 194, 196, 231, 234]  # nibble kernel on the WorkQueue grid (fused_nb.hpp)

CRC = sorted(set(CRC_STREAM + XOR_FUSED + RS_FUSED))
