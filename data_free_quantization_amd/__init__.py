"""MI355X-native DFQ weight-transform path (data-free quantization, Nagel et al.
ICCV'19, as implemented by KadAMRN/Data_Free_Quantization).

Host layer mirrors the reference's module APIs; the arithmetic runs in
libdfq_hip.so (hand-written HIP for gfx950, C ABI in include/dfq_hip.h):

    from data_free_quantization_amd.utils.quantize import quantize
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm, quantize_targ_layer
    from data_free_quantization_amd.utils.relation import create_relation
    from data_free_quantization_amd.Cross_layer_equal import cross_layer_equalization
    from data_free_quantization_amd.bias_absorption import bias_absorption
    from data_free_quantization_amd.clip_weight import clip_weight
    from data_free_quantization_amd.bias_correction import bias_correction
"""
__version__ = "0.1.0"
