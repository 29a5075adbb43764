"""``paddle.text.datasets`` parsers over the archives the reference downloads (no network here:
each dataset reads a local ``data_file`` with the same member layout and produces the same
samples). Reference: `python/paddle/text/datasets/{imdb,imikolov,movielens,conll05,wmt14,wmt16}.py`.

* ``Imdb``: aclImdb tar — documents tokenised (trailing newlines stripped, ASCII punctuation
  removed, lower-cased, whitespace split); vocabulary = words seen more than ``cutoff`` times in
  train + test, ordered by (−count, word), ``<unk>`` last; samples (word ids, [label]) with pos = 0,
  neg = 1.
* ``Imikolov``: PTB ``simple-examples`` tar — vocabulary from train + valid counts (each line adds
  one ``<s>`` and one ``<e>``), words seen more than ``min_word_freq`` times, ``<unk>`` last;
  ``NGRAM`` windows of ``<s> … <e>`` or ``SEQ`` (src = ``<s>`` + ids, trg = ids + ``<e>``).
* ``Movielens``: ml-1m zip — user (id, gender, age bucket, job), movie (id, category ids, title
  word ids), rating·2 − 5; a seeded uniform draw per rating assigns it to train or test.
* ``Conll05st``: CoNLL-2005 test.wsj words / props (gzip members of the tar) + word / verb /
  label dictionaries: one sample per predicate of a sentence with the ±2 predicate context words,
  the predicate mark and BIO labels.
* ``WMT14``: tar with ``*src.dict`` / ``*trg.dict`` (first ``dict_size`` lines) and
  ``{mode}/{mode}`` tab-separated pairs; pairs with > 80 ids dropped.
* ``WMT16``: ``wmt16/{train,test,val}``; dictionaries built from the train split's counts
  (``<s> <e> <unk>`` first) and cached next to the archive.
"""
from __future__ import annotations

import collections
import gzip
import io
import os
import re
import string
import tarfile
import zipfile

import numpy as np

from ..io import Dataset

_PUNCT = str.maketrans("", "", string.punctuation)


def _need(data_file, name):
    if data_file is None:
        raise RuntimeError(f"{name}: no network access in this environment; pass data_file= (the "
                           "reference archive)")
    return data_file


def _text(b):
    return b.decode("utf-8", errors="replace") if isinstance(b, bytes) else b


def _vocab(counts, min_count, drop=()):
    items = [(w, c) for w, c in counts.items() if c > min_count and w not in drop]
    items.sort(key=lambda wc: (-wc[1], wc[0]))
    idx = {w: i for i, (w, _) in enumerate(items)}
    idx["<unk>"] = len(items)
    return idx


class Imdb(Dataset):
    def __init__(self, data_file=None, mode="train", cutoff=150, download=True):
        assert mode.lower() in ("train", "test"), mode
        self.mode = mode.lower()
        self.data_file = _need(data_file, "Imdb")
        both = re.compile(r"aclImdb/(train|test)/(pos|neg)/.*\.txt$")
        counts = collections.Counter()
        for doc in self._docs(both):
            counts.update(doc)
        self.word_idx = _vocab(counts, cutoff)
        unk = self.word_idx["<unk>"]
        self.docs, self.labels = [], []
        for label, pol in ((0, "pos"), (1, "neg")):
            for doc in self._docs(re.compile(rf"aclImdb/{self.mode}/{pol}/.*\.txt$")):
                self.docs.append([self.word_idx.get(w, unk) for w in doc])
                self.labels.append(label)

    def _docs(self, pattern):
        with tarfile.open(self.data_file) as tf:
            for m in tf:
                if m.isfile() and pattern.match(m.name):
                    raw = tf.extractfile(m).read().rstrip(b"\n\r")
                    yield _text(raw).translate(_PUNCT).lower().split()

    def __getitem__(self, i):
        return np.array(self.docs[i]), np.array([self.labels[i]])

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    def __init__(self, data_file=None, data_type="NGRAM", window_size=-1, mode="train", min_word_freq=50,
                 download=True):
        self.data_type = data_type.upper()
        assert self.data_type in ("NGRAM", "SEQ"), data_type
        assert mode.lower() in ("train", "test", "valid"), mode
        self.mode = mode.lower()
        self.window_size = window_size
        self.data_file = _need(data_file, "Imikolov")
        counts = collections.Counter()
        for split in ("train", "valid"):
            for line in self._lines(split):
                counts.update(line.split())
                counts["<s>"] += 1
                counts["<e>"] += 1
        self.word_idx = _vocab(counts, min_word_freq, drop=("<unk>",))
        unk = self.word_idx["<unk>"]
        split = "valid" if self.mode == "test" and not self._has("test") else self.mode
        self.data = []
        for line in self._lines(split):
            words = line.split()
            if self.data_type == "NGRAM":
                assert window_size > -1, "NGRAM needs window_size"
                ids = [self.word_idx.get(w, unk) for w in ["<s>"] + words + ["<e>"]]
                self.data += [tuple(ids[i - window_size:i]) for i in range(window_size, len(ids) + 1)]
            else:
                ids = [self.word_idx.get(w, unk) for w in words]
                src = [self.word_idx["<s>"]] + ids
                if window_size > 0 and len(src) > window_size:
                    continue
                self.data.append((src, ids + [self.word_idx["<e>"]]))

    def _member(self, split):
        return f"./simple-examples/data/ptb.{split}.txt"

    def _has(self, split):
        with tarfile.open(self.data_file) as tf:
            names = tf.getnames()
        return self._member(split) in names or self._member(split)[2:] in names

    def _lines(self, split):
        with tarfile.open(self.data_file) as tf:
            names = set(tf.getnames())
            name = self._member(split)
            if name not in names:
                name = name[2:]
            for raw in tf.extractfile(name):
                yield _text(raw).strip()

    def __getitem__(self, i):
        return tuple(np.array(d) for d in self.data[i])

    def __len__(self):
        return len(self.data)


_AGES = [1, 18, 25, 35, 45, 50, 56]


class Movielens(Dataset):
    def __init__(self, data_file=None, mode="train", test_ratio=0.1, rand_seed=0, download=True):
        assert mode.lower() in ("train", "test"), mode
        self.mode = mode.lower()
        self.data_file = _need(data_file, "Movielens")
        np.random.seed(rand_seed)
        title_re = re.compile(r"^(.*)\((\d+)\)$")
        movies, users = {}, {}
        titles, cats = [], []
        with zipfile.ZipFile(self.data_file) as z:
            for raw in z.open("ml-1m/movies.dat"):
                mid, title, cat = raw.decode("latin").strip().split("::")
                title = title_re.match(title).group(1)
                movies[int(mid)] = (int(mid), cat.split("|"), title)
                for w in title.split():
                    if w.lower() not in titles:
                        titles.append(w.lower())
                for c in cat.split("|"):
                    if c not in cats:
                        cats.append(c)
            self.movie_title_dict = {w: i for i, w in enumerate(titles)}
            self.categories_dict = {c: i for i, c in enumerate(cats)}
            for raw in z.open("ml-1m/users.dat"):
                uid, g, age, job, _ = raw.decode("latin").strip().split("::")
                users[int(uid)] = (int(uid), 0 if g == "M" else 1, _AGES.index(int(age)), int(job))
            self.data = []
            want_test = self.mode == "test"
            for raw in z.open("ml-1m/ratings.dat"):
                if (np.random.random() < test_ratio) != want_test:
                    continue
                uid, mid, r, _ = raw.decode("latin").strip().split("::")
                u, m = users[int(uid)], movies[int(mid)]
                self.data.append([[u[0]], [u[1]], [u[2]], [u[3]], [m[0]],
                                  [self.categories_dict[c] for c in m[1]],
                                  [self.movie_title_dict[w.lower()] for w in m[2].split()],
                                  [float(r) * 2 - 5.0]])

    def __getitem__(self, i):
        return tuple(np.array(d) for d in self.data[i])

    def __len__(self):
        return len(self.data)


class Conll05st(Dataset):
    UNK_IDX = 0

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None,
                 emb_file=None, download=True):
        self.data_file = _need(data_file, "Conll05st")
        for f, n in ((word_dict_file, "word_dict_file"), (verb_dict_file, "verb_dict_file"),
                     (target_dict_file, "target_dict_file")):
            _need(f, f"Conll05st {n}")
        self.emb_file = emb_file
        self.word_dict = self._dict(word_dict_file)
        self.predicate_dict = self._dict(verb_dict_file)
        self.label_dict = self._label_dict(target_dict_file)
        self.sentences, self.predicates, self.labels = [], [], []
        self._parse()

    @staticmethod
    def _dict(path):
        with open(path) as f:
            return {line.strip(): i for i, line in enumerate(f)}

    @staticmethod
    def _label_dict(path):
        tags = []
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line[:2] in ("B-", "I-") and line[2:] not in tags:
                    tags.append(line[2:])
        d = {}
        for t in tags:
            d["B-" + t] = len(d)
            d["I-" + t] = len(d)
        d["O"] = len(d)
        return d

    @staticmethod
    def _bio(column):
        out, tag, open_ = [], "O", False
        for t in column:
            if t == "*":
                out.append("I-" + tag if open_ else "O")
            elif t == "*)":
                out.append("I-" + tag)
                open_ = False
            elif "(" in t:
                tag = t[1:t.find("*")]
                out.append("B-" + tag)
                open_ = ")" not in t
            else:
                raise RuntimeError(f"Conll05st: unexpected label {t!r}")
        return out

    def _parse(self):
        with tarfile.open(self.data_file) as tf:
            wraw = tf.extractfile("conll05st-release/test.wsj/words/test.wsj.words.gz").read()
            praw = tf.extractfile("conll05st-release/test.wsj/props/test.wsj.props.gz").read()
        words = gzip.GzipFile(fileobj=io.BytesIO(wraw))
        props = gzip.GzipFile(fileobj=io.BytesIO(praw))
        sent, rows = [], []
        for w, p in zip(words, props):
            w, cols = _text(w).strip(), _text(p).strip().split()
            if cols:
                sent.append(w)
                rows.append(cols)
                continue
            if rows:  # end of sentence: column 0 = predicates, 1.. = one argument labelling each
                ncol = len(rows[0])
                verbs = [r[0] for r in rows if r[0] != "-"]
                for j in range(1, ncol):
                    self.sentences.append(list(sent))
                    self.predicates.append(verbs[j - 1])
                    self.labels.append(self._bio([r[j] for r in rows]))
            sent, rows = [], []

    def __getitem__(self, i):
        s, pred, lab = self.sentences[i], self.predicates[i], self.labels[i]
        n = len(s)
        v = lab.index("B-V")
        mark = [0] * n
        ctx = {}
        for off, name, edge in ((-2, "n2", "bos"), (-1, "n1", "bos"), (0, "0", None), (1, "p1", "eos"),
                                (2, "p2", "eos")):
            j = v + off
            if 0 <= j < n:
                mark[j] = 1
                ctx[name] = s[j]
            else:
                ctx[name] = edge
        wi = lambda w: self.word_dict.get(w, self.UNK_IDX)  # noqa: E731
        rep = lambda w: np.array([wi(w)] * n)  # noqa: E731
        return (np.array([wi(w) for w in s]), rep(ctx["n2"]), rep(ctx["n1"]), rep(ctx["0"]), rep(ctx["p1"]),
                rep(ctx["p2"]), np.array([self.predicate_dict.get(pred)] * n), np.array(mark),
                np.array([self.label_dict.get(t) for t in lab]))

    def __len__(self):
        return len(self.sentences)

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return self.emb_file


class WMT14(Dataset):
    START, END, UNK, UNK_IDX = "<s>", "<e>", "<unk>", 2

    def __init__(self, data_file=None, mode="train", dict_size=-1, download=True):
        assert mode.lower() in ("train", "test", "gen"), mode
        assert dict_size > 0, "dict_size should be set as positive number"
        self.mode = mode.lower()
        self.data_file = _need(data_file, "WMT14")
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        with tarfile.open(self.data_file) as tf:
            names = tf.getnames()

            def dict_of(suffix):
                (name,) = [n for n in names if n.endswith(suffix)]
                d = {}
                for i, raw in enumerate(tf.extractfile(name)):
                    if i >= dict_size:
                        break
                    d[_text(raw).strip()] = i
                return d
            self.src_dict, self.trg_dict = dict_of("src.dict"), dict_of("trg.dict")
            for name in [n for n in names if n.endswith(f"{self.mode}/{self.mode}")]:
                for raw in tf.extractfile(name):
                    parts = _text(raw).strip().split("\t")
                    if len(parts) != 2:
                        continue
                    src = [self.src_dict.get(w, self.UNK_IDX) for w in [self.START] + parts[0].split() + [self.END]]
                    trg = [self.trg_dict.get(w, self.UNK_IDX) for w in parts[1].split()]
                    if len(src) > 80 or len(trg) > 80:
                        continue
                    self.src_ids.append(src)
                    self.trg_ids.append([self.trg_dict[self.START]] + trg)
                    self.trg_ids_next.append(trg + [self.trg_dict[self.END]])

    def __getitem__(self, i):
        return np.array(self.src_ids[i]), np.array(self.trg_ids[i]), np.array(self.trg_ids_next[i])

    def __len__(self):
        return len(self.src_ids)

    def get_dict(self, reverse=False):
        if reverse:
            return ({v: k for k, v in self.src_dict.items()}, {v: k for k, v in self.trg_dict.items()})
        return self.src_dict, self.trg_dict


class WMT16(Dataset):
    MARKS = ("<s>", "<e>", "<unk>")

    def __init__(self, data_file=None, mode="train", src_dict_size=-1, trg_dict_size=-1, lang="en",
                 download=True):
        assert mode.lower() in ("train", "test", "val"), mode
        assert src_dict_size > 0 and trg_dict_size > 0, "dict sizes should be positive"
        self.mode, self.lang = mode.lower(), lang
        self.data_file = _need(data_file, "WMT16")
        self.src_dict = self._dict(lang, src_dict_size)
        self.trg_dict = self._dict("de" if lang == "en" else "en", trg_dict_size)
        s, e, u = (self.src_dict[m] for m in self.MARKS)
        sc = 0 if lang == "en" else 1
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        for a, b in self._pairs(self.mode):
            src, trg = (a, b) if sc == 0 else (b, a)
            self.src_ids.append([s] + [self.src_dict.get(w, u) for w in src.split()] + [e])
            t = [self.trg_dict.get(w, u) for w in trg.split()]
            self.trg_ids.append([s] + t)
            self.trg_ids_next.append(t + [e])

    def _pairs(self, split):
        with tarfile.open(self.data_file) as tf:
            for raw in tf.extractfile(f"wmt16/{split}"):
                parts = _text(raw).strip().split("\t")
                if len(parts) == 2:
                    yield parts

    def _dict(self, lang, size):
        """<s> <e> <unk> then the train split's words of ``lang`` by descending count; cached as
        ``<archive dir>/wmt16_<lang>_<size>.dict``."""
        path = os.path.join(os.path.dirname(os.path.abspath(self.data_file)), f"wmt16_{lang}_{size}.dict")
        words = None
        if os.path.exists(path):
            with open(path, encoding="utf-8") as f:
                words = [w.rstrip("\n") for w in f]
            if len(words) != size:
                words = None
        if words is None:
            counts = collections.Counter()
            col = 0 if lang == "en" else 1
            for pair in self._pairs("train"):
                counts.update(pair[col].split())
            ranked = sorted(counts.items(), key=lambda wc: wc[1], reverse=True)
            words = list(self.MARKS) + [w for w, _ in ranked][:max(0, size - 3)]
            try:
                with open(path, "w", encoding="utf-8") as f:
                    f.write("\n".join(words) + "\n")
            except OSError:
                pass
        return {w: i for i, w in enumerate(words)}

    def __getitem__(self, i):
        return np.array(self.src_ids[i]), np.array(self.trg_ids[i]), np.array(self.trg_ids_next[i])

    def __len__(self):
        return len(self.src_ids)

    def get_dict(self, lang, reverse=False):
        d = self.src_dict if lang == self.lang else self.trg_dict
        return {v: k for k, v in d.items()} if reverse else d
