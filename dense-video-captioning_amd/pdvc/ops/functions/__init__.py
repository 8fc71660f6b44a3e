from .ms_deform_attn_func import (MSDeformAttnFunction, ms_deform_attn_core_pytorch, MSDA1dFunction, NUM_SAMPLES_FUSED,
                                  CapGatherFunction)
from .caption_decode import CaptionDecodeFunction
from .linear import LinearFunction, dense, matmul
from .addnorm import AddDropoutLayerNormFunction, add_dropout_layernorm
