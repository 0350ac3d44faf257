"""Training / evaluation dataset with the glyph layout on the GPU (SURVEY.md 8(f) row 2;
reference: scripts/dataset.py:13-202, scripts/utils/tools.py:22-72,585-635,
scripts/04_train.py:47-58).

Same constructor, ``__getitem__`` keys, ``collate_fn`` (sort by text length, split the
batch_size x group_size loader batch into batch_size groups, optional tail) and 13-item
batch tuple as the reference.  What moves: the reference centres every character of the
rendered strip into a ``max_pixelsize``-wide white cell with cv2/numpy per sample in the
DataLoader workers, pads the batch with ``pad_2D_gray_image`` and converts with
``ToTensor`` on the host.  Here a sample carries its raw strip and per-character widths;
``reprocess`` puts them in a :class:`GlyphBatch`, and ``utils.tools.to_device`` lays the
whole batch out on the GPU in one ``vo_glyph_batch`` launch -- the host does no per-pixel
work, which is what keeps 8 data-parallel ranks fed.  PNG decoding uses PIL (cv2 is not a
dependency of this package).
"""

import json
from pathlib import Path

import numpy as np
from torch.utils.data import Dataset as _TorchDataset

from .utils.symbols import get_symbols
from .utils.tools import pad_1D, pad_2D


class GlyphBatch:
    """Raw grayscale strips (H, W_b) uint8 and their per-character widths for one batch.
    ``to(device)`` -> (B, 1, H, W) fp32 laid out exactly as the reference's
    character_padding_forinput + pad_2D_gray_image + ToTensor (bit-identical)."""

    def __init__(self, strips, char_widths, cell, stride):
        self.strips = [np.ascontiguousarray(s, dtype=np.uint8) for s in strips]
        self.char_widths = [np.asarray(w, np.int64).reshape(-1) for w in char_widths]
        self.cell, self.stride = int(cell), int(stride)

    def __len__(self):
        return len(self.strips)

    @property
    def margin(self):
        return (self.stride // 2) * self.cell  # pad_2D_gray_image's each_padlen

    def to(self, device):
        from . import ops
        return ops.glyph_batch(self.strips, self.char_widths, self.cell, self.margin, device)


def _read_gray(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("L"), dtype=np.uint8)


class Dataset(_TorchDataset):
    def __init__(self, filename, preprocess_config, train_config, model_config, sort=False, drop_last=False):
        self.preprocessed_path = Path(preprocess_config["path"]["preprocessed"])
        self.batch_size = train_config["optimizer"]["batch_size"]
        self.input_type = preprocess_config["input_type"]
        self.symbol_to_id = get_symbols(self.preprocessed_path)
        self.sort = sort
        self.drop_last = drop_last
        self.use_image = train_config["use_image"]
        self.is_energy = model_config["variance_embedding"]["is_energy_condition"]
        self.is_kurtosis = model_config["variance_embedding"]["is_kurtosis_condition"]
        if self.input_type == "visual-text":
            vt = preprocess_config["visual_text"]
            self.text_font_size = vt["fontsize"]
            self.image_bgcolor = vt["color"]["background"]
            self.image_textcolor = vt["color"]["text"]
            self.image_loadscale = vt["scale_in_training"]
            if self.image_loadscale != "gray-scale":
                raise NotImplementedError("RGB glyph input: the reference's pad_2D_image path is not on the "
                                          "ICASSP configuration")
            with open(self.preprocessed_path / "visual_text.json") as f:
                info = json.load(f)
            self.width = info["max_pixelsize"][0]
            self.height = info["height"][0]
            self.stride = vt["stride"]
        self.basename, self.audiotype, self.fontsize, self.fonttype, self.text = self.process_meta(filename)
        with open(self.preprocessed_path / "audiotype.json") as f:
            self.audiotype_map = json.load(f)

    def __len__(self):
        return len(self.text)

    def __getitem__(self, idx):
        basename = self.basename[idx]
        audiotype = self.audiotype[idx]
        tmp_text = self.text[idx].replace("{", "").replace("}", "").replace("\n", "")
        text = np.array([self.symbol_to_id[t] for t in list(tmp_text)])
        p = self.preprocessed_path
        mel = np.load(p / "mel" / audiotype / f"{basename}.npy")
        energy = np.load(p / "energy" / audiotype / f"{basename}.npy") if self.is_energy else None
        kurtosis = np.load(p / "kurtosis" / audiotype / f"{basename}.npy") if self.is_kurtosis else None
        duration = np.load(p / "duration" / audiotype / f"{basename}.npy")
        image = None
        if self.use_image:
            widths = np.load(p / "image" / "width" / audiotype / f"{basename}.npy").astype(np.int32)
            if np.max(widths) > self.width:
                print(f"image length is over {self.width} pixels. {basename}")
            image = (_read_gray(p / "image" / "png" / audiotype / f"{basename}.png"), widths)
        return {"id": basename, "audiotype": self.audiotype_map[audiotype], "text": text, "mel": mel,
                "energy": energy, "kurtosis": kurtosis, "duration": duration, "image": image,
                "event_image_feature": None}

    def process_meta(self, filename):
        names, audiotypes, fonttypes, fontsizes, texts = [], [], [], [], []
        with open(self.preprocessed_path / filename, "r", encoding="utf-8") as f:
            for line in f.readlines():
                fn, at, fs, ft, r = line.strip("\n").split("|")
                names.append(fn)
                audiotypes.append(at)
                fonttypes.append(ft)
                fontsizes.append(fs)
                texts.append(r)
        return names, audiotypes, fonttypes, fontsizes, texts

    def reprocess(self, data, idxs):
        ids = [data[i]["id"] for i in idxs]
        audiotypes = np.array([data[i]["audiotype"] for i in idxs])
        texts = [data[i]["text"] for i in idxs]
        mels = [data[i]["mel"] for i in idxs]
        energies = [data[i]["energy"] for i in idxs]
        kurtosises = [data[i]["kurtosis"] for i in idxs]
        durations = [data[i]["duration"] for i in idxs]
        text_lens = np.array([t.shape[0] for t in texts])
        mel_lens = np.array([m.shape[0] for m in mels])
        texts = pad_1D(texts)
        mels = pad_2D(mels)
        energies = pad_1D(energies) if energies[0] is not None else None
        kurtosises = pad_1D(kurtosises) if kurtosises[0] is not None else None
        durations = pad_1D(durations)
        images = None
        if self.use_image:
            images = GlyphBatch([data[i]["image"][0] for i in idxs], [data[i]["image"][1] for i in idxs],
                                self.width, self.stride)
        event_image_features = np.array([data[i]["event_image_feature"] for i in idxs])
        return (ids, audiotypes, texts, text_lens, max(text_lens), mels, mel_lens, max(mel_lens), energies,
                kurtosises, durations, images, event_image_features)

    def collate_fn(self, data):
        n = len(data)
        if self.sort:
            idx_arr = np.argsort(-np.array([d["text"].shape[0] for d in data]))
        else:
            idx_arr = np.arange(n)
        tail = idx_arr[len(idx_arr) - (len(idx_arr) % self.batch_size):]
        idx_arr = idx_arr[: len(idx_arr) - (len(idx_arr) % self.batch_size)]
        idx_arr = idx_arr.reshape((-1, self.batch_size)).tolist()
        if not self.drop_last and len(tail) > 0:
            idx_arr += [tail.tolist()]
        return [self.reprocess(data, idx) for idx in idx_arr]
