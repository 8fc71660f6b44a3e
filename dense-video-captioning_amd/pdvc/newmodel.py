"""NewModel (reference: NewModel.py:9-94) -- PDVC behind the dual-modality front-end, for cfgs/yc2_newModel_sound.yml.

Same attribute names as the reference (pdvcModel, pdvcCriterion, pdvcPostprocessor, ln1, mha1, mlp_seq1, ln2, mha2,
mlp_seq2), so the front-end and PDVC state_dict keys match; the reference's `sound_model` (HuBERT, downloaded by
torchaudio at construction) is not part of this model: the per-clip sound features come in through
dt['sound_tensor'] (N, T, 768), as they do in the reference once cached (NewModel.py:98-100).  The reference reads
one video's TSP features and audio from disk inside forward (get_vid_features / get_mfcc); here both arrive in the
batch: dt['video_tensor'] (N, T, 768) clips and dt['sound_tensor'].  forward returns (output, loss, 0) as the
reference's does (`los` is always 0 there, NewModel.py:76,93).
"""
from torch import nn

from pdvc.frontend import DualModalityFrontEnd
from pdvc.pdvc import build


class NewModel(DualModalityFrontEnd):
    def __init__(self, args, dim=768, num_heads=32):
        super().__init__(dim, num_heads)
        self.pdvcModel, self.pdvcCriterion, self.pdvcPostprocessor = build(args)
        self.args = args

    def forward(self, dt, eval_mode=False):
        dt = dict(dt)
        dt["video_tensor"] = super().forward(dt["video_tensor"], dt.pop("sound_tensor"))
        output, loss = self.pdvcModel(dt, self.pdvcCriterion, self.args.transformer_input_type, eval_mode=eval_mode)
        return output, loss, 0


class NewModelStep(nn.Module):
    """A NewModel behind PDVC's calling convention, model(dt, criterion, transformer_input_type, eval_mode) ->
    (output, loss) (pdvc.py:124), so the training-step machinery (StepGraph, bench.py) drives it like PDVC:
    the front-end runs on dt['video_tensor'] / dt['sound_tensor'], then PDVC on its output."""

    def __init__(self, newmodel):
        super().__init__()
        self.newmodel = newmodel

    def forward(self, dt, criterion=None, transformer_input_type="queries", eval_mode=False):
        m = self.newmodel
        clips = dt["video_tensor"]
        # the front-end output replaces the clips for PDVC only while it runs: dt stays the caller's object (PDVC
        # caches its host-side facts in it, which a hipGraph capture of the step relies on) and keeps the clips
        dt["video_tensor"] = DualModalityFrontEnd.forward(m, clips, dt["sound_tensor"])
        try:
            return m.pdvcModel(dt, criterion if criterion is not None else m.pdvcCriterion, transformer_input_type,
                               eval_mode=eval_mode)
        finally:
            dt["video_tensor"] = clips


def build_newmodel(args):
    """(model, criterion, postprocessors) like pdvc.build, with the front-end in front (NewModel.py:15)."""
    m = NewModel(args)
    return m, m.pdvcCriterion, {"bbox": m.pdvcPostprocessor}
