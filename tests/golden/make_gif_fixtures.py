"""Decode the reference's recorded games (docs/ GIFs) into JSON fixtures.

Run here (never on the GPU box): `python tests/golden/make_gif_fixtures.py`. It reads the
animated GIFs the reference ships under /root/reference/docs/images/AlphaZero/ — frames rendered
by `ColosseumBlokusGameWrapper.render` (blokus_rl/colossumrl/blokus_wrapper.py:248-279) from
real colosseumrl games — and writes, per game, the ordered list of placements
(colour, [[row, col], ...]) to tests/golden/gif_<name>.json. Those files are data (inputs and
expected outputs); no reference source is copied.

Decoding (matplotlib defaults of render()): 640x480 frames, axes span
x in [80, 576] px and y in [57.6, 427.2] px, board cell (row=y, col=x) sampled at pixel
(427.2 - (y+0.5)*369.6/N, 80 + (x+0.5)*496/N); nearest colour of
{0 lightgrey, 1 red, 2 blue, 3 yellow, 4 green} (blokus_wrapper.py:259).
"""
import json
import os
import sys

import numpy as np
from PIL import Image, ImageSequence

REF_DOCS = "/root/reference/docs/images/AlphaZero"
HERE = os.path.dirname(os.path.abspath(__file__))

PALETTE = {
    0: (211, 211, 211),
    1: (255, 0, 0),
    2: (0, 0, 255),
    3: (255, 255, 0),
    4: (0, 128, 0),
}

GAMES = {
    "arena20": ("blokus_20/arena.gif", 20, 4),
    "win7": ("blokus_7/step_1_win.gif", 7, 2),
    "draw7": ("blokus_7/step_104_draw.gif", 7, 2),
}


def decode_frame(img: Image.Image, n: int) -> np.ndarray:
    rgb = np.asarray(img.convert("RGB")).astype(np.int32)
    h, w, _ = rgb.shape
    sy, sx = h / 480.0, w / 640.0
    board = np.zeros((n, n), dtype=np.int8)
    cols = np.array([PALETTE[k] for k in range(5)])
    for y in range(n):
        for x in range(n):
            py = int(round((427.2 - (y + 0.5) * 369.6 / n) * sy))
            px = int(round((80 + (x + 0.5) * 496 / n) * sx))
            c = rgb[py, px]
            board[y, x] = int(np.argmin(((cols - c) ** 2).sum(axis=1)))
    return board


def decode_game(path: str, n: int):
    frames = [decode_frame(f, n) for f in ImageSequence.Iterator(Image.open(path))]
    placements = []
    prev = frames[0]
    assert (prev == 0).all(), "first frame must be the empty board"
    for fr in frames[1:]:
        diff = (fr != prev)
        if not diff.any():
            continue  # duplicated frame
        assert (prev[diff] == 0).all(), "a frame overwrote a placed cell"
        colours = set(int(v) for v in fr[diff])
        assert len(colours) == 1, f"a frame added several colours: {colours}"
        cells = sorted([int(r), int(c)] for r, c in zip(*np.nonzero(diff)))
        placements.append({"colour": colours.pop(), "cells": cells})
        prev = fr
    return placements, prev


def main():
    for name, (rel, n, p) in GAMES.items():
        path = os.path.join(REF_DOCS, rel)
        placements, final = decode_game(path, n)
        squares = [int((final == k + 1).sum()) for k in range(p)]
        out = {
            "source": f"reference docs/images/AlphaZero/{rel}",
            "board_size": n,
            "num_players": p,
            "placements": placements,
            "final_squares": squares,
        }
        fp = os.path.join(HERE, f"gif_{name}.json")
        with open(fp, "w", encoding="utf-8") as f:
            json.dump(out, f, indent=1)
        print(f"{name}: {len(placements)} placements, squares {squares} -> {fp}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
