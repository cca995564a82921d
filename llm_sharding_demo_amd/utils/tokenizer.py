"""Tokenizers.

The reference calls `AutoTokenizer.from_pretrained(MODEL_ID)` in every role
(`server.py:40`), which needs the HF Hub at boot.  Here:
  * if a local directory with GPT-2 `vocab.json` + `merges.txt` (or a
    `tokenizer.json`) is available (TOKENIZER_PATH, or the weights dir), the
    real byte-level BPE is used via the `tokenizers` library;
  * otherwise a byte-level fallback maps each UTF-8 byte to the id GPT-2's
    vocab gives that byte's unicode stand-in (the bytes_to_unicode table,
    [tf5.15] convert_slow_tokenizer.py:1879), so fallback ids remain valid,
    decodable GPT-2 ids.  Ids the fallback cannot map back to a byte decode
    to a visible placeholder.
`decode(..., skip_special_tokens=True)` mirrors `server.py:209`.
"""
from __future__ import annotations

import os
from typing import List, Optional


def bytes_to_unicode_order() -> List[int]:
    """Byte values in GPT-2 vocab order: vocab id k <-> byte bs[k] for k < 256."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    for b in range(256):
        if b not in bs:
            bs.append(b)
    return bs


class ByteTokenizer:
    name = "byte-fallback"

    def __init__(self, gpt2_ids: bool = True, eos_id: Optional[int] = 50256):
        order = bytes_to_unicode_order() if gpt2_ids else list(range(256))
        self.byte_to_id = {b: i for i, b in enumerate(order)}
        self.id_to_byte = {i: b for i, b in enumerate(order)}
        self.eos_id = eos_id

    def encode(self, text: str) -> List[int]:
        return [self.byte_to_id[b] for b in text.encode("utf-8")]

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out = bytearray()
        parts: List[str] = []
        for i in ids:
            i = int(i)
            if i in self.id_to_byte:
                out.append(self.id_to_byte[i])
                continue
            if skip_special_tokens and i == self.eos_id:
                continue
            parts.append(out.decode("utf-8", errors="replace"))
            out = bytearray()
            parts.append(f"<{i}>")
        parts.append(out.decode("utf-8", errors="replace"))
        return "".join(parts)


class BPETokenizer:
    name = "bpe"

    def __init__(self, path: str):
        from tokenizers import Tokenizer

        tj = os.path.join(path, "tokenizer.json")
        if os.path.isfile(tj):
            self.tok = Tokenizer.from_file(tj)
        else:
            from tokenizers import ByteLevelBPETokenizer

            self.tok = ByteLevelBPETokenizer(os.path.join(path, "vocab.json"),
                                             os.path.join(path, "merges.txt"))
        self.special = {v for k, v in self.tok.get_vocab().items() if k.startswith("<|")}

    def encode(self, text: str) -> List[int]:
        return self.tok.encode(text).ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        ids = [int(i) for i in ids]
        if skip_special_tokens:
            ids = [i for i in ids if i not in self.special]
        return self.tok.decode(ids, skip_special_tokens=skip_special_tokens)


def load_tokenizer(model_id: str, arch: str = "gpt2", weights: Optional[str] = None,
                   eos_id: Optional[int] = None):
    for path in (os.environ.get("TOKENIZER_PATH"), weights, model_id):
        if path and os.path.isdir(path) and (
                os.path.isfile(os.path.join(path, "tokenizer.json")) or
                (os.path.isfile(os.path.join(path, "vocab.json")) and
                 os.path.isfile(os.path.join(path, "merges.txt")))):
            return BPETokenizer(path)
    return ByteTokenizer(gpt2_ids=(arch == "gpt2"), eos_id=eos_id)
