"""``paddle.text`` datasets (`text/datasets.py`) on small synthetic archives laid out like the
reference downloads (aclImdb tar, PTB simple-examples tar, ml-1m zip, CoNLL-2005 test.wsj tar +
dictionaries, WMT14 / WMT16 tars): vocabulary rules, sample layouts and split handling of the
reference parsers (`python/paddle/text/datasets/*.py`)."""
import gzip
import io
import tarfile
import zipfile

import numpy as np

from paddle_infer_amd import text


def _tar(path, members, mode="w:gz"):
    with tarfile.open(path, mode) as tf:
        for name, data in members.items():
            data = data.encode() if isinstance(data, str) else data
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    return str(path)


def test_imdb(tmp_path):
    m = {"aclImdb/train/pos/0.txt": "Good movie, good!\n", "aclImdb/train/neg/0.txt": "Bad. bad movie",
         "aclImdb/test/pos/0.txt": "good good", "aclImdb/test/neg/1.txt": "bad film"}
    f = _tar(tmp_path / "imdb.tgz", m)
    ds = text.Imdb(data_file=f, mode="train", cutoff=1)
    # counts over train+test: good 5, bad 3, movie 2, film 1 → kept (>1): good, bad, movie
    assert ds.word_idx == {"good": 0, "bad": 1, "movie": 2, "<unk>": 3}
    assert len(ds) == 2
    doc, lab = ds[0]
    np.testing.assert_array_equal(doc, [0, 2, 0]) and np.testing.assert_array_equal(lab, [0])
    np.testing.assert_array_equal(ds[1][0], [1, 1, 2])
    assert ds[1][1][0] == 1
    te = text.Imdb(data_file=f, mode="test", cutoff=1)
    np.testing.assert_array_equal(te[1][0], [1, 3])


def test_imikolov(tmp_path):
    m = {"./simple-examples/data/ptb.train.txt": "a b c\na b\n", "./simple-examples/data/ptb.valid.txt": "a c\n",
         "./simple-examples/data/ptb.test.txt": "b c d\n"}
    f = _tar(tmp_path / "ptb.tgz", m)
    ng = text.Imikolov(data_file=f, data_type="NGRAM", window_size=3, mode="train", min_word_freq=1)
    # counts: <s> 3, <e> 3, a 3, b 2, c 2 → all kept (>1), ordered (-count, word)
    assert ng.word_idx == {"<e>": 0, "<s>": 1, "a": 2, "b": 3, "c": 4, "<unk>": 5}
    assert [int(v) for v in ng[0]] == [1, 2, 3]
    assert ng.data[:3] == [(1, 2, 3), (2, 3, 4), (3, 4, 0)]
    sq = text.Imikolov(data_file=f, data_type="SEQ", mode="test", min_word_freq=1)
    src, trg = sq[0]
    np.testing.assert_array_equal(src, [1, 3, 4, 5])
    np.testing.assert_array_equal(trg, [3, 4, 5, 0])


def test_movielens(tmp_path):
    p = tmp_path / "ml-1m.zip"
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("ml-1m/movies.dat", "1::Toy Story (1995)::Animation|Comedy\n2::Heat (1995)::Action\n")
        z.writestr("ml-1m/users.dat", "1::F::1::10::48067\n2::M::25::7::70072\n")
        z.writestr("ml-1m/ratings.dat", "".join(f"{u}::{m}::{r}::0\n" for u, m, r in
                                                [(1, 1, 5), (1, 2, 3), (2, 1, 4), (2, 2, 1)] * 5))
    tr = text.Movielens(data_file=str(p), mode="train", test_ratio=0.3, rand_seed=1)
    te = text.Movielens(data_file=str(p), mode="test", test_ratio=0.3, rand_seed=1)
    assert len(tr) + len(te) == 20 and len(te) > 0
    s = tr[0]
    assert len(s) == 8 and s[-1].dtype == np.float64
    uid = int(s[0][0])
    assert int(s[1][0]) == (1 if uid == 1 else 0) and int(s[2][0]) == (0 if uid == 1 else 2)
    assert set(tr.categories_dict) == {"Animation", "Comedy", "Action"}
    assert float(s[-1][0]) in (5.0, 1.0, 3.0, -3.0)


def test_conll05(tmp_path):
    words = "The\ncat\nsat\ndown\n\n"
    props = "-\t(A0*\nsat\t*)\n-\t(V*)\n-\t(AM-DIR*)\n\n".replace("\t", " ")
    m = {"conll05st-release/test.wsj/words/test.wsj.words.gz": gzip.compress(words.encode()),
         "conll05st-release/test.wsj/props/test.wsj.props.gz": gzip.compress(props.encode())}
    f = _tar(tmp_path / "conll.tgz", m)
    (tmp_path / "w.txt").write_text("<unk>\nThe\ncat\nsat\ndown\nbos\neos\n")
    (tmp_path / "v.txt").write_text("sat\n")
    (tmp_path / "t.txt").write_text("B-A0\nI-A0\nB-V\nI-V\nB-AM-DIR\nI-AM-DIR\nO\n")
    ds = text.Conll05st(data_file=f, word_dict_file=str(tmp_path / "w.txt"), verb_dict_file=str(tmp_path / "v.txt"),
                        target_dict_file=str(tmp_path / "t.txt"))
    assert len(ds) == 1 and ds.labels[0] == ["B-A0", "I-A0", "B-V", "B-AM-DIR"]
    w, n2, n1, c0, p1, p2, pred, mark, lab = ds[0]
    np.testing.assert_array_equal(w, [1, 2, 3, 4])
    assert n2[0] == 1 and n1[0] == 2 and c0[0] == 3 and p1[0] == 4 and p2[0] == 6
    np.testing.assert_array_equal(mark, [1, 1, 1, 1])
    np.testing.assert_array_equal(pred, [0] * 4)
    ld = ds.label_dict
    np.testing.assert_array_equal(lab, [ld["B-A0"], ld["I-A0"], ld["B-V"], ld["B-AM-DIR"]])


def test_wmt14(tmp_path):
    m = {"wmt14/src.dict": "<s>\n<e>\n<unk>\nhello\nworld\n", "wmt14/trg.dict": "<s>\n<e>\n<unk>\nhallo\nwelt\n",
         "wmt14/train/train": "hello world\thallo welt\nhello\thallo\nbad line\n"}
    ds = text.WMT14(data_file=_tar(tmp_path / "wmt14.tgz", m), mode="train", dict_size=4)
    assert len(ds) == 2
    src, trg, nxt = ds[0]
    np.testing.assert_array_equal(src, [0, 3, 2, 1])      # "world" beyond dict_size → <unk>=2
    np.testing.assert_array_equal(trg, [0, 3, 2])
    np.testing.assert_array_equal(nxt, [3, 2, 1])


def test_wmt16(tmp_path):
    m = {"wmt16/train": "a b a\tx y\nb\ty y\n", "wmt16/test": "a c\tx z\n"}
    f = _tar(tmp_path / "wmt16.tgz", m)
    ds = text.WMT16(data_file=f, mode="test", src_dict_size=5, trg_dict_size=4, lang="en")
    assert ds.src_dict == {"<s>": 0, "<e>": 1, "<unk>": 2, "a": 3, "b": 4}
    assert ds.trg_dict == {"<s>": 0, "<e>": 1, "<unk>": 2, "y": 3}
    src, trg, nxt = ds[0]
    np.testing.assert_array_equal(src, [0, 3, 2, 1])
    np.testing.assert_array_equal(trg, [0, 2, 2])
    np.testing.assert_array_equal(nxt, [2, 2, 1])
