"""LEAF Shakespeare character pipeline (reference: ``data/shakespeare/language_utils.py:29-41``,
``data/shakespeare/data_loader.py:53-63``).

LEAF stores each client's samples as 80-character strings (``x``) and the next character (``y``).
Characters map to indices in the TFF text-generation vocabulary (the vocabulary is dataset
definition, shared with the reference so trained models agree on token ids). The reference maps an
unknown character to ``str.find``'s -1, which its embedding cannot index; here it maps to the OOV id
(``len(ALL_LETTERS)``, one of the 4 extra ids of ``VOCAB_SIZE``). The model (``RNN_OriginalFedAvg``,
last-step logits, classification CE) embeds ``VOCAB_SIZE`` = 90 ids."""
from typing import List, Sequence

import numpy as np

# TFF "Federated Learning for Text Generation" character vocabulary (data, not code)
CHAR_VOCAB = list("dhlptx@DHLPTX $(,048cgkoswCGKOSW[_#'/37;?bfjnrvzBFJNRVZ\"&*.26:\naeimquyAEIMQUY]!%)-159\r")
ALL_LETTERS = "".join(CHAR_VOCAB)
VOCAB_SIZE = len(ALL_LETTERS) + 4     # + OOV, padding (0), BOS, EOS
_INDEX = {ch: i for i, ch in enumerate(ALL_LETTERS)}


OOV_ID = len(ALL_LETTERS)


def letter_to_index(letter: str) -> int:
    return _INDEX.get(letter, OOV_ID)


def word_to_indices(word: str) -> List[int]:
    return [_INDEX.get(ch, OOV_ID) for ch in word]


def letter_to_vec(letter: str) -> List[int]:
    v = [0] * VOCAB_SIZE
    v[letter_to_index(letter)] = 1
    return v


def process_x(raw_x_batch: Sequence[str]) -> np.ndarray:
    """[n] strings of equal length → int64 [n, L] character ids."""
    return np.asarray([word_to_indices(w) for w in raw_x_batch], dtype=np.int64)


def process_y(raw_y_batch: Sequence[str]) -> np.ndarray:
    return np.asarray([letter_to_index(c) for c in raw_y_batch], dtype=np.int64)


def is_char_data(values) -> bool:
    """LEAF text clients store strings; image/feature clients store numbers."""
    return len(values) > 0 and isinstance(values[0], str)
