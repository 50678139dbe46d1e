"""Tokenizers and chat templates.

No network is available, so the real Llama-3 (tiktoken BPE) and BERT
WordPiece vocabularies cannot be downloaded.  Two implementations share one
interface:

* ``ByteTokenizer`` -- UTF-8 bytes map to ids 0..255 of the model vocabulary;
  the model's special tokens keep their real ids (Llama-3 <|begin_of_text|>
  128000, <|eot_id|> 128009, ...).  Ids >= 256 produced by a random-weight
  model detokenize to a printable character so streamed output stays valid
  UTF-8.  Token counts equal byte counts, which makes synthetic prompt
  lengths exact.
* ``HFTokenizer`` -- wraps a local ``tokenizer.json`` (the `tokenizers`
  library) when real weights are served.

The chat template reproduces Llama-3's header/eot format.  The reference
flattens messages to "role: content" lines for Ollama generate
(core/internal/routing/router.go:379, MessagesToPrompt); that flattening is
kept in ``messages_to_prompt`` for the job API.
"""
from __future__ import annotations

from pathlib import Path

LLAMA3_SPECIAL = {
    "<|begin_of_text|>": 128000, "<|end_of_text|>": 128001,
    "<|start_header_id|>": 128006, "<|end_header_id|>": 128007,
    "<|eom_id|>": 128008, "<|eot_id|>": 128009,
}


class ByteTokenizer:
    def __init__(self, vocab_size: int, special: dict[str, int] | None = None,
                 bos: int | None = None, eos: tuple[int, ...] = ()):
        self.vocab_size = vocab_size
        self.special = dict(special or {})
        self.id_to_special = {v: k for k, v in self.special.items()}
        self.bos_id = bos
        self.eos_ids = tuple(eos)

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = list(text.encode("utf-8"))
        return ([self.bos_id] if add_bos and self.bos_id is not None else []) + ids

    def token_bytes(self, tid: int) -> bytes:
        if 0 <= tid < 256:
            return bytes([tid])
        if tid in self.id_to_special:
            return b""
        return bytes([32 + tid % 95])  # printable stand-in for non-byte ids

    def decode(self, ids, skip_special: bool = True) -> str:
        out = bytearray()
        for t in ids:
            if not skip_special and t in self.id_to_special:
                out += self.id_to_special[t].encode()
            else:
                out += self.token_bytes(int(t))
        return out.decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str | Path, bos: int | None = None, eos: tuple[int, ...] = ()):
        from tokenizers import Tokenizer  # local file only
        p = Path(path)
        if p.is_dir():
            p = p / "tokenizer.json"
        self.tok = Tokenizer.from_file(str(p))
        self.vocab_size = self.tok.get_vocab_size()
        self.bos_id = bos
        self.eos_ids = tuple(eos)
        self.special = {k: v for k, v in self.tok.get_vocab().items()
                        if k.startswith("<|") and k.endswith("|>")}

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] if add_bos and self.bos_id is not None else []) + ids

    def token_bytes(self, tid: int) -> bytes:
        return self.tok.decode([tid], skip_special_tokens=True).encode("utf-8")

    def decode(self, ids, skip_special: bool = True) -> str:
        return self.tok.decode(list(map(int, ids)), skip_special_tokens=skip_special)


class IncrementalDetokenizer:
    """Streams text deltas without splitting UTF-8 sequences, and detects stop
    strings (OpenAI ``stop``) across token boundaries."""

    def __init__(self, tok, stop: list[str] | None = None):
        self.tok = tok
        self.buf = bytearray()
        self.text = ""
        self.stop = [s for s in (stop or []) if s]
        self.stopped = False

    def push(self, tid: int) -> str:
        if self.stopped:
            return ""
        self.buf += self.tok.token_bytes(tid)
        try:
            piece = self.buf.decode("utf-8")
            self.buf.clear()
        except UnicodeDecodeError as e:
            if len(self.buf) - e.start > 3:  # invalid, not just incomplete
                piece = self.buf.decode("utf-8", errors="replace")
                self.buf.clear()
            else:
                piece = self.buf[: e.start].decode("utf-8")
                del self.buf[: e.start]
        if not piece:
            return ""
        prev = len(self.text)
        self.text += piece
        if self.stop:
            lo = max(0, prev - max(len(s) for s in self.stop))
            cut = -1
            for s in self.stop:
                i = self.text.find(s, lo)
                if i >= 0 and (cut < 0 or i < cut):
                    cut = i
            if cut >= 0:
                self.stopped = True
                delta = self.text[prev:cut] if cut >= prev else ""
                self.text = self.text[:cut]
                return delta
        return piece

    def flush(self) -> str:
        if self.stopped or not self.buf:
            return ""
        piece = self.buf.decode("utf-8", errors="replace")
        self.buf.clear()
        self.text += piece
        return piece


def apply_chat_template(tok, messages: list[dict], add_generation_prompt: bool = True,
                        family: str = "llama") -> list[int]:
    """Llama-3 chat format:
    <|begin_of_text|>(<|start_header_id|>role<|end_header_id|>\\n\\ncontent<|eot_id|>)*
    <|start_header_id|>assistant<|end_header_id|>\\n\\n"""
    sp = getattr(tok, "special", {}) or {}
    bot = sp.get("<|begin_of_text|>")
    sh, eh, eot = sp.get("<|start_header_id|>"), sp.get("<|end_header_id|>"), sp.get("<|eot_id|>")
    ids: list[int] = []
    if sh is None or eh is None or eot is None:
        # model without chat specials: plain "role: content" lines
        return tok.encode(messages_to_prompt(messages) + ("\nassistant:" if add_generation_prompt
                                                          else ""), add_bos=True)
    if bot is not None:
        ids.append(bot)
    for m in messages:
        ids.append(sh)
        ids += tok.encode(str(m.get("role", "user")))
        ids.append(eh)
        ids += tok.encode("\n\n" + _content_text(m.get("content", "")))
        ids.append(eot)
    if add_generation_prompt:
        ids.append(sh)
        ids += tok.encode("assistant")
        ids.append(eh)
        ids += tok.encode("\n\n")
    return ids


def _content_text(c) -> str:
    if isinstance(c, str):
        return c
    if isinstance(c, list):  # OpenAI content parts
        return "".join(p.get("text", "") for p in c if isinstance(p, dict))
    return "" if c is None else str(c)


def messages_to_prompt(messages: list[dict]) -> str:
    """Reference flattening (router.go:379-391): one 'role: content' line per
    message; messages with neither role nor content are skipped."""
    lines = []
    for m in messages or []:
        content = _content_text(m.get("content", ""))
        if not m.get("role") and not content:
            continue
        role = m.get("role") or "user"
        lines.append(f"{role}: {content}")
    return "\n".join(lines)


def for_model(cfg, tokenizer_path: str | None = None):
    eos = tuple(getattr(cfg, "eos_token_ids", ()) or ())
    bos = getattr(cfg, "bos_token_id", None)
    if tokenizer_path:
        return HFTokenizer(tokenizer_path, bos=bos, eos=eos)
    if getattr(cfg, "family", "") == "llama" and cfg.vocab_size >= 128256:
        return ByteTokenizer(cfg.vocab_size, LLAMA3_SPECIAL, bos=128000, eos=eos)
    if getattr(cfg, "family", "") == "nomic-bert":
        return ByteTokenizer(cfg.vocab_size, {"[CLS]": 101, "[SEP]": 102}, bos=101, eos=(102,))
    # tiny test models: specials at the top of the vocab
    V = cfg.vocab_size
    special = {"<|begin_of_text|>": V - 6, "<|end_of_text|>": V - 5,
               "<|start_header_id|>": V - 4, "<|end_header_id|>": V - 3, "<|eot_id|>": V - 2}
    return ByteTokenizer(V, special, bos=V - 6, eos=tuple(eos) + (V - 2,))
