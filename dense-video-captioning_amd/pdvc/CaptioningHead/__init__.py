"""Caption heads (reference: pdvc/CaptioningHead/__init__.py:5-21).  'standard' (LSTM + deformable soft
attention) is the head of every BASELINE config; 'light' and 'none' are outside this build's scope
 and raise."""
from .LSTM_DSA import LSTMDSACaptioner


def build_captioner(opt):
    if opt.caption_decoder_type == "standard":
        opt.event_context_dim = None
        opt.clip_context_dim = opt.hidden_dim
        return LSTMDSACaptioner(opt)
    if opt.caption_decoder_type in ("light", "none"):
        raise NotImplementedError(f"caption_decoder_type '{opt.caption_decoder_type}' is not part of the MI355X "
                                  f"hot path (use 'standard')")
    raise ValueError("caption decoder type is invalid")
