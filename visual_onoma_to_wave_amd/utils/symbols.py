"""Vocabulary (reference: scripts/utils/symbols.py:4-17): the sorted set of characters of
train/val/test.txt, ids from 1 (0 = PAD).  When the split files are absent (no corpus
offline) the packaged ``symbols.json`` of the same directory layout is used."""

import json
import os


def get_symbols(preprocess_path):
    names = ["train.txt", "val.txt", "test.txt"]
    if all(os.path.exists(os.path.join(preprocess_path, n)) for n in names):
        chars = set()
        for n in names:
            with open(os.path.join(preprocess_path, n), "r", encoding="utf-8") as f:
                for line in f:
                    text = line.strip("\n").split("|")[4]
                    chars.update(text.replace("{", "").replace("}", ""))
        seq = sorted(chars)
    else:
        with open(os.path.join(preprocess_path, "symbols.json"), encoding="utf-8") as f:
            seq = json.load(f)
    return {s: i + 1 for i, s in enumerate(seq)}
