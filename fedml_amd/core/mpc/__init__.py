from .finite_field import (DEFAULT_PRIME, BGW_decoding, BGW_encoding, Gen_Additive_SS, LCC_decoding,
                           LCC_decoding_with_points, LCC_encoding, LCC_encoding_w_Random,
                           LCC_encoding_w_Random_partial, LCC_encoding_with_points, PI, additive_share,
                           dequantize_from_field, divmod, gen_BGW_lambda_s, gen_Lagrange_coeffs, mod_matmul,
                           modular_inv, my_key_agreement, my_pk_gen, quantize_to_field)
from .secagg import SecureAggregator, SecAggClient, pairwise_mask
