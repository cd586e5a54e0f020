"""Tokenizers: the real HF ``tokenizer.json`` when present, a synthetic twin otherwise.

No network is available, so the published Qwen3 / Mistral tokenizer files
cannot be fetched.  When a model directory (``BCG_WEIGHTS``/``BCG_TOKENIZER``)
holds a ``tokenizer.json`` it is used as-is.  Otherwise we build a
*synthetic* byte-level BPE with the same vocabulary size, the same special
tokens (ids and spelling) and the Qwen2 pre-tokenizer regex, trained
deterministically on text that ships with the image (Python stdlib + site
packages sources).  It tokenises the BCG prompts at ~3.6 chars/token (the
real Qwen tokenizer: ~4), which keeps prefill/decode shapes and the
guided-decoding mask work representative.  Results produced with it are
labelled "synthetic tokenizer" by the benchmark.

Reproducibility: the trained files ship with the package
(``engine/assets/synthetic-<family>-v1.json.gz``) and their SHA-256 is pinned
below (``PINNED_SHA256``), so every box -- whatever its site-packages --
tokenises identically.  Only when an asset is missing is the tokenizer
re-trained from the image's text corpus (cached in ``<repo>/.cache/tokenizers``,
concurrent processes serialise on a lock file); a re-trained file whose hash
differs from the pin is refused unless ``BCG_ALLOW_UNPINNED_TOKENIZER=1``.
"""

import fcntl
import glob
import gzip
import hashlib
import json
import os
from functools import lru_cache
from typing import Dict, List, Optional

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CACHE_DIR = os.environ.get("BCG_TOKENIZER_CACHE", os.path.join(REPO, ".cache", "tokenizers"))
ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")

# sha256 of the (uncompressed) synthetic tokenizer JSON every result was produced with
PINNED_SHA256 = {
    "qwen": "49bafd542f956b0e25607fa604a39aaaec17304fa3e7e507e1675ee4408f2ff2",
    "mistral": "78a20091e6e5007467688e582b23fcaff114a5b879b108b29d4d2090eac6ce99",
}

QWEN_PATTERN = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                r"|\s*[\r\n]+|\s+(?!\S)|\s+")

QWEN_SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>", "<|object_ref_start|>",
                 "<|object_ref_end|>", "<|box_start|>", "<|box_end|>", "<|quad_start|>", "<|quad_end|>",
                 "<|vision_start|>", "<|vision_end|>", "<|vision_pad|>", "<|image_pad|>", "<|video_pad|>",
                 "<tool_call>", "</tool_call>", "<|fim_prefix|>", "<|fim_middle|>", "<|fim_suffix|>",
                 "<|fim_pad|>", "<|repo_name|>", "<|file_sep|>", "<tool_response>", "</tool_response>",
                 "<think>", "</think>"]
MISTRAL_SPECIALS = ["<unk>", "<s>", "</s>", "[INST]", "[/INST]", "[TOOL_CALLS]", "[AVAILABLE_TOOLS]",
                    "[/AVAILABLE_TOOLS]", "[TOOL_RESULTS]", "[/TOOL_RESULTS]"]

FAMILIES = {
    # family: (regular BPE vocab, specials, specials first?, eos tokens)
    "qwen": (151643, QWEN_SPECIALS, False, ["<|im_end|>", "<|endoftext|>"]),
    "mistral": (32768 - len(MISTRAL_SPECIALS), MISTRAL_SPECIALS, True, ["</s>"]),
}


def _bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


BYTE_TO_UNI = _bytes_to_unicode()
UNI_TO_BYTE = {v: k for k, v in BYTE_TO_UNI.items()}


def _corpus_files(limit_bytes: int = 150_000_000) -> List[str]:
    files = sorted(glob.glob("/usr/lib/python3.10/**/*.py", recursive=True))
    site = "/usr/local/lib/python3.10/dist-packages"
    files += sorted(glob.glob(f"{site}/**/*.md", recursive=True))
    files += sorted(glob.glob(f"{site}/**/*.py", recursive=True))
    out, total = [], 0
    for f in files:
        try:
            size = os.path.getsize(f)
        except OSError:
            continue
        if total + size > limit_bytes:
            break
        out.append(f)
        total += size
    return out


def _train_synthetic(family: str, path: str):
    n_regular, specials, specials_first, _ = FAMILIES[family]
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(QWEN_PATTERN), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(
        vocab_size=n_regular + (len(specials) if specials_first else 0),
        min_frequency=2, show_progress=False,
        initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
        special_tokens=specials if specials_first else [])

    def texts():
        for f in _corpus_files():
            with open(f, encoding="utf-8", errors="ignore") as fh:
                yield fh.read()

    tok.train_from_iterator(texts(), trainer)
    if not specials_first:
        tok.add_special_tokens(specials)
    else:
        tok.add_special_tokens(specials)  # mark them special (ids already assigned)
    tmp = path + f".tmp{os.getpid()}"
    tok.save(tmp)
    os.replace(tmp, path)


class BCGTokenizer:
    """Thin wrapper exposing what the engine needs (encode/decode/token bytes/EOS)."""

    def __init__(self, tok: Tokenizer, eos_tokens: List[str], synthetic: bool, name: str):
        self.tok = tok
        self.synthetic = synthetic
        self.name = name
        self.vocab_size = tok.get_vocab_size(with_added_tokens=True)
        self.eos_token_ids = [i for i in (tok.token_to_id(t) for t in eos_tokens) if i is not None]
        self.eos_token_id = self.eos_token_ids[0] if self.eos_token_ids else None
        added = tok.get_added_tokens_decoder() if hasattr(tok, "get_added_tokens_decoder") else {}
        self.special_ids = {i for i, t in added.items() if getattr(t, "special", True)}

    def encode(self, text: str) -> List[int]:
        return self.tok.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self.tok.encode_batch(texts, add_special_tokens=False)]

    def encode_batch_safe(self, texts: List[str]):
        """encode_batch for text that may hold lone UTF-16 surrogates (a JSON ``\\ud83d`` escape
        json.loads accepts, quoted back into a later prompt): the tokenizer refuses such a string,
        and with it the whole batch.  Those characters become U+FFFD instead.  Returns (ids, the
        number of texts that needed it)."""
        try:
            return self.encode_batch(texts), 0
        except (TypeError, ValueError, UnicodeError):
            fixed = [encodable(t) for t in texts]
            return self.encode_batch(fixed), sum(a is not b for a, b in zip(fixed, texts))

    def decode(self, ids: List[int]) -> str:
        return self.tok.decode(ids, skip_special_tokens=True)

    def decode_bytes(self, ids: List[int]) -> bytes:
        return b"".join(self.token_bytes(i) for i in ids)

    @lru_cache(maxsize=None)
    def token_bytes(self, i: int) -> bytes:
        if i in self.special_ids:
            return b""
        piece = self.tok.id_to_token(i)
        if piece is None:
            return b""
        if all(ch in UNI_TO_BYTE for ch in piece):
            return bytes(UNI_TO_BYTE[ch] for ch in piece)
        # sentencepiece-style vocab (real Mistral/Llama files)
        if piece.startswith("<0x") and piece.endswith(">") and len(piece) == 6:
            return bytes([int(piece[3:5], 16)])
        return piece.replace("▁", " ").encode("utf-8")

    def all_token_bytes(self) -> List[bytes]:
        return [self.token_bytes(i) for i in range(self.vocab_size)]


def encodable(text: str) -> str:
    """`text` with every lone surrogate replaced by U+FFFD (the same object when it has none)."""
    try:
        text.encode("utf-8")
        return text
    except UnicodeEncodeError:
        return "".join("\ufffd" if 0xD800 <= ord(c) <= 0xDFFF else c for c in text)


def family_of(model_name: str) -> str:
    low = model_name.lower()
    return "mistral" if ("mistral" in low or "llama" in low) else "qwen"


_CACHE: Dict[str, BCGTokenizer] = {}


def load_tokenizer(model_name: str, model_dir: Optional[str] = None) -> BCGTokenizer:
    key = f"{model_name}|{model_dir}"
    if key in _CACHE:
        return _CACHE[key]
    family = family_of(model_name)
    eos = FAMILIES[family][3]
    for d in filter(None, [model_dir, os.environ.get("BCG_TOKENIZER")]):
        path = d if d.endswith(".json") else os.path.join(d, "tokenizer.json")
        if os.path.exists(path):
            tok = BCGTokenizer(Tokenizer.from_file(path), eos, synthetic=False, name=path)
            _CACHE[key] = tok
            return tok
    tok = BCGTokenizer(Tokenizer.from_str(synthetic_json(family)), eos, synthetic=True,
                       name=f"synthetic-{family}")
    _CACHE[key] = tok
    return tok


def synthetic_json(family: str) -> str:
    """The pinned synthetic tokenizer of `family` (shipped asset, else re-trained + verified)."""
    asset = os.path.join(ASSET_DIR, f"synthetic-{family}-v1.json.gz")
    if os.path.exists(asset):
        with gzip.open(asset, "rb") as fh:
            raw = fh.read()
        source = asset
    else:
        os.makedirs(CACHE_DIR, exist_ok=True)
        path = os.path.join(CACHE_DIR, f"synthetic-{family}-v1.json")
        if not os.path.exists(path):
            with open(path + ".lock", "w") as lock:
                fcntl.flock(lock, fcntl.LOCK_EX)
                if not os.path.exists(path):
                    _train_synthetic(family, path)
                fcntl.flock(lock, fcntl.LOCK_UN)
        with open(path, "rb") as fh:
            raw = fh.read()
        source = path
    digest = hashlib.sha256(raw).hexdigest()
    if digest != PINNED_SHA256[family] and os.environ.get("BCG_ALLOW_UNPINNED_TOKENIZER") != "1":
        raise RuntimeError(f"synthetic {family} tokenizer {source} has sha256 {digest}, pinned "
                           f"{PINNED_SHA256[family]}: results would not be comparable "
                           "(set BCG_ALLOW_UNPINNED_TOKENIZER=1 to use it anyway)")
    return raw.decode("utf-8")
