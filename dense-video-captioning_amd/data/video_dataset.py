"""Real-data ingestion for PDVC training (reference: data/video_dataset.py).

What a user of the reference's `data.video_dataset` imports, with the same names and behaviour:

  * `collate_fn(batch)`            per-video tuples -> the flat `dt` dict PDVC.forward reads (:15-149);
  * `Translator(json, vocab_size)` caption <-> token ids (:152-180);
  * `PropSeqDataset(anno, folders, vocab_json, is_training, proposal_type, opt)` (:223-293): loads each
    video's features, rescales them to `frame_embedding_num` rows, subsamples at most
    `gt_proposal_sample_num` events (numpy's global RNG, as the reference), tokenises the captions;
  * `resizeFeature(x, n, 'nearest')` (:386-397), `get_feats` / `read_file` (:315-383).

`resizeFeature` is scipy's interp1d(kind='nearest') on the grid i*(T-1)/(n-1), restated as a row gather:
row i takes source row k = #{midpoints m + 0.5 < x_i} (ties round down, as interp1d's searchsorted), so the
result is bit-identical and keeps the input dtype.  `resize_rows_device` is the same gather for features
already in HBM (one index_select per video).

Feature files: .npy (numpy.load, pickles refused) and .csv (pandas).  The reference also unpickles .pkl
files; that executes code from the file and is refused here (ValueError).  Missing files give zero
features of 100 rows and the padding flag, as in the reference.
"""
import json
import os
from collections import defaultdict

import numpy as np
from torch.utils.data import Dataset

from pdvc.data import collate

# keyed by visual_feature_type: feature width, normalisation constants, file name from the video key
_FEATURE_TYPES = {
    "c3d": (500, -0.001915027447565527, 1.9239444588254049, lambda k: k[0:13] + ".npy"),
    "resnet": (2048, 0.41634243404998694, 0.2569392081183313, lambda k: k[2:13] + "_resnet.npy"),
    "bn": (1024, 0.8945046635916155, 3.6579982046018844, lambda k: k[2:13] + "_bn.npy"),
    "tsn_100": (400, 0, 0, lambda k: k[0:13] + ".csv"),
    "i3d_rgb": (1024, 0, 0, lambda k: k[:13] + "_rgb.npy"),
    "i3d_flow": (1024, 0, 0, lambda k: k[:13] + "_flow.npy"),
    "tsp": (512, 0, 0, lambda k: k[0:13] + ".npy"),
    "tsp_mvit": (768, 0, 0, lambda k: k[0:13] + ".npy"),
    "vggish": (128, 0, 0, lambda k: k[0:13] + ".npy"),
}

# punctuation the reference blanks out before splitting a sentence into words (video_dataset.py:164)
_PUNCT = [",", ":", "!", "_", ";", "-", ".", "?", "/", '"', "\\n", "\\", "."]


def collate_fn(batch):
    """Per-video tuples (feature (T, C), featstamps, labels, captions, timestamps, duration, raw captions,
    key) -> the `dt` dict; videos are zero-padded to the longest and masked (pdvc/data.py:collate)."""
    return collate(batch)


class Translator:
    """Vocabulary JSON {"word_to_ix": {...}, "ix_to_word": {...}} of `vocab_size` words.  Unknown words
    translate to id `vocab_size`."""

    def __init__(self, translator_json, vocob_size):
        with open(translator_json) as f:
            vocab = json.load(f)
        self._init(vocab, vocob_size)

    @classmethod
    def from_vocab(cls, ix_to_word):
        """A translator built from an in-memory ix_to_word mapping {str(id): word}."""
        tr = cls.__new__(cls)
        tr._init({"ix_to_word": dict(ix_to_word), "word_to_ix": {w: int(i) for i, w in ix_to_word.items()}},
                 len(ix_to_word))
        return tr

    def _init(self, vocab, vocab_size):
        self.vocab_size = vocab_size
        if vocab_size != len(vocab["word_to_ix"]):
            raise AssertionError(f"vocabulary has {len(vocab['word_to_ix'])} words, vocab_size is {vocab_size}")
        self.vocab = {"word_to_ix": defaultdict(lambda: self.vocab_size, vocab["word_to_ix"]),
                      "ix_to_word": defaultdict(lambda: self.vocab_size, vocab["ix_to_word"])}

    def translate(self, sentence, max_len):
        """[0] + word ids (at most max_len - 2) + [0]."""
        for p in _PUNCT:
            sentence = sentence.replace(p, " ")
        words = sentence.lower().split()
        w2i = self.vocab["word_to_ix"]
        return np.array([0] + [w2i[w] for w in words][:max_len - 2] + [0])

    def rtranslate_batch(self, seqs, yield_every=0):
        """rtranslate of every row of an int array (R, L), in one native pass (pdvc_detokenize: the first-zero
        cut, the word lookup and the joins in C, one byte buffer for all rows)."""
        from pdvc import _native
        seqs = np.asarray(seqs)
        if seqs.size == 0:
            return [""] * seqs.shape[0]
        tab = getattr(self, "_word_table", None)
        if tab is None or tab[2] <= int(seqs.max()):
            i2w = self.vocab["ix_to_word"]
            n = max(int(seqs.max()) + 1, len(i2w) + 1)
            enc = [b""] + [i2w[str(i)].encode("utf-8") if str(i) in i2w else None for i in range(1, n)]
            if any(e is None for e in enc[1:int(seqs.max()) + 1]):
                missing = next(i for i in range(1, int(seqs.max()) + 1) if enc[i] is None)
                raise KeyError(str(missing))  # as rtranslate: an id without a word
            enc = [e if e is not None else b"" for e in enc]
            off = np.zeros(n + 1, np.int64)
            off[1:] = np.cumsum([len(e) for e in enc])
            tab = (np.frombuffer(b"".join(enc), dtype=np.uint8).copy(), off, n)
            self._word_table = tab
        return _native.detokenize(seqs.astype(np.int64, copy=False), tab[0], tab[1], yield_every)

    def rtranslate(self, sent_ids):
        """Ids up to the first 0 -> 'w1 w2 ... wn.' ('' when the caption is empty)."""
        ids = list(sent_ids)
        if 0 in ids:
            ids = ids[:ids.index(0)]
        if not ids:
            return ""
        i2w = self.vocab["ix_to_word"]
        return " ".join(i2w[str(i)] for i in ids) + "."


def nearest_rows(original_size, new_size):
    """Source row of every output row of interp1d(arange(T), ., kind='nearest') at i*(T-1)/(n-1)."""
    x_new = np.asarray([i * float(original_size - 1) / (new_size - 1) for i in range(new_size)])
    midpoints = (np.arange(1, original_size) + np.arange(original_size - 1)) / 2.0
    return np.clip(np.searchsorted(midpoints, x_new, side="left"), 0, original_size - 1)


def resizeFeature(inputData, newSize, sample_method="nearest"):
    """(T, C) features -> (newSize, C) by nearest-neighbour resampling; a single row is repeated."""
    if sample_method != "nearest":
        raise NotImplementedError(f"resizeFeature: sample_method {sample_method!r} (the reference uses 'nearest')")
    x = np.asarray(inputData)
    if len(x) == 1:
        return np.stack([x.reshape(-1)] * newSize)
    return x[nearest_rows(len(x), newSize)]


def resize_rows_device(features, new_size):
    """resizeFeature for a (T, C) tensor already on the device: one row gather."""
    import torch
    idx = torch.as_tensor(nearest_rows(features.shape[0], new_size), device=features.device)
    if features.shape[0] == 1:
        return features.reshape(1, -1).expand(new_size, -1).contiguous()
    return features.index_select(0, idx)


def read_file(path, feat_dim, MEAN=0.0, VAR=1.0, data_norm=False):
    """Feature matrix of one file and whether it was missing (zero padding, 100 rows)."""
    if os.path.exists(path):
        ext = path.split(".")[-1]
        if ext == "npy":
            feats = np.load(path, allow_pickle=False)
        elif ext == "csv":
            import pandas as pd
            feats = pd.read_csv(path).values
        elif ext == "pkl":
            raise ValueError(f"{path}: pickled feature files are not loaded (unpickling executes code)")
        else:
            raise NotImplementedError(ext)
        padding = False
    else:
        print("{} not exists, use zero padding. ".format(path))
        feats = np.zeros((100, feat_dim))
        padding = True
    if data_norm:
        feats = (feats - MEAN) / np.sqrt(VAR)
    return feats, padding


def get_feats(key, vf_type, vf_folder, data_norm=False):
    if vf_type not in _FEATURE_TYPES:
        raise AssertionError("feature type error")
    feat_dim, mean, var, name = _FEATURE_TYPES[vf_type]
    path = os.path.join(vf_folder, name(key))
    feats, padding = read_file(path, feat_dim, mean, var, data_norm)
    if len(feats.shape) == 1:
        assert feats.shape[0] == feat_dim, "load {} error, got shape {}".format(path, feats.shape)
    assert feats.shape[1] == feat_dim, "load {} error, got shape {}".format(path, feats.shape)
    return feats, padding


class EDVCdataset(Dataset):
    def __init__(self, anno_file, feature_folder, translator_json, is_training, proposal_type, opt):
        super().__init__()
        with open(anno_file) as f:
            self.anno = json.load(f)
        self.translator = Translator(translator_json, opt.vocab_size)
        self.max_caption_len = opt.max_caption_len
        self.keys = list(self.anno.keys())
        for json_path in opt.invalid_video_json:
            with open(json_path) as f:
                invalid = json.load(f)
            self.keys = [k for k in self.keys if k[:13] not in invalid]
        self.feature_folder = feature_folder
        self.feature_sample_rate = opt.feature_sample_rate
        self.opt = opt
        self.proposal_type = proposal_type
        self.is_training = is_training
        self.train_proposal_sample_num = opt.train_proposal_sample_num
        self.gt_proposal_sample_num = opt.gt_proposal_sample_num
        self.feature_dim = opt.feature_dim
        self.num_queries = opt.num_queries

    def __len__(self):
        return len(self.keys)

    @staticmethod
    def process_time_step(duration, timestamps_list, feature_length):
        """Event timestamps (s) -> integer feature indices in [0, feature_length - 1]."""
        stamps = feature_length * np.array(timestamps_list) / np.array(duration)
        stamps = np.minimum(stamps, np.array(feature_length) - 1).astype("int")
        return np.maximum(stamps, 0).astype("int").tolist()


class PropSeqDataset(EDVCdataset):
    def load_feats(self, key):
        vf_types = self.opt.visual_feature_type
        if isinstance(vf_types, list):  # several feature types: each rescaled, then concatenated
            if not (isinstance(self.feature_folder, list) and len(vf_types) == len(self.feature_folder)):
                raise AssertionError("one feature folder per visual_feature_type")
            parts = []
            all_padding = True
            for vf_type, vf_folder in zip(vf_types, self.feature_folder):
                feats, is_padding = get_feats(key, vf_type, vf_folder)
                all_padding = is_padding & all_padding
                if self.opt.data_rescale:
                    if feats.shape[0] != self.opt.frame_embedding_num:
                        feats = resizeFeature(feats, self.opt.frame_embedding_num, "nearest")
                else:
                    feats = feats[::self.opt.feature_sample_rate]
                parts.append(feats)
            if all_padding:
                print("all feature files of video {} do not exist".format(key))
            out = np.concatenate(parts, axis=-1)
        else:
            out, _ = get_feats(key, vf_types, self.feature_folder, data_norm=self.opt.data_norm)
            if self.opt.data_rescale:
                out = resizeFeature(out, self.opt.frame_embedding_num, "nearest")
        assert out.shape[1] == self.feature_dim, "wrong value of feature_dim"
        return out

    def __getitem__(self, idx):
        key = str(self.keys[idx])
        feats = self.load_feats(key)
        a = self.anno[key]
        duration, captions, stamps = a["duration"], a["sentences"], a["timestamps"]
        labels = a.get("action_labels", [0] * len(stamps))
        assert max(labels) <= self.opt.num_classes
        n = min(len(stamps), self.gt_proposal_sample_num)
        keep = set(np.random.choice(list(range(len(stamps))), n, replace=False).tolist())
        captions = [c for i, c in enumerate(captions) if i in keep]
        stamps = [s for i, s in enumerate(stamps) if i in keep]
        labels = [lab for i, lab in enumerate(labels) if i in keep]
        tokens = [np.array(self.translator.translate(s, self.max_caption_len)) for s in captions]
        featstamps = self.process_time_step(duration, stamps, feats.shape[0])
        return feats, featstamps, labels, tokens, stamps, duration, captions, key
