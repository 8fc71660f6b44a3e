from .ms_deform_attn import MSDeformAttn
from .ms_deform_attn_for_caption import MSDeformAttnCap
