"""nn.Linear with the same parameters and state_dict names whose forward runs on pdvc_gemm_f32
(ops/functions/linear.py: `dense`); `forward(x, relu=True)` fuses the ReLU of an FFN's first layer."""
from torch import nn

from ..functions.linear import dense


class Linear(nn.Linear):
    def forward(self, x, relu=False):
        return dense(x, self.weight, self.bias, relu)
