"""Token ids of the text vocabulary (same values as the reference's transformer/Constants.py)."""
PAD, UNK, BOS, EOS = 0, 1, 2, 3
PAD_WORD, UNK_WORD, BOS_WORD, EOS_WORD = "<blank>", "<unk>", "<s>", "</s>"
