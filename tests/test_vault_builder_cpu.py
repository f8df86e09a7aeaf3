"""Truth-Vault index builder (mmf_amd.vault_builder, train_clip_detective.py:457-607) on CPU:
the reference's pickle schema and skip-on-error behaviour, and the sharded build over a
world-size-2 gloo group (one all-gather) equal to the single-process build.  The encoder here is
the CPU oracle's CLIP (test infrastructure); on the GPU the HIP towers (tests/test_gpu_api.py)."""
import json
import os
import pickle
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
N_ART = 9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _articles(tmp):
    """N_ART articles with synthetic images on disk; article 4 points at a missing file."""
    from PIL import Image
    import mmf_amd.synthetic as syn
    imgs = syn.images(N_ART, 55)
    ids, _ = syn.clip_ids(N_ART, 77, 56, [77, 20, 5, 60, 9, 33, 2, 70, 15])
    lens = [77, 20, 5, 60, 9, 33, 2, 70, 15]
    arts, table = [], {}
    for i in range(N_ART):
        p = os.path.join(tmp, f"a{i}.png")
        if i != 4:
            Image.fromarray(imgs[i]).save(p)
        text = f"article text {i}"
        table[text] = ids[i, :lens[i]].tolist()
        arts.append({"article_id": f"id{i}", "text_content": text, "image_local_path": p})
    with open(os.path.join(tmp, "seed.json"), "w") as f:
        json.dump(arts, f)
    return arts, table


def _oracle_encoder():
    import mmf_amd.weights as W
    from oracle import models as M
    clip = M.to_torch(W.synthetic_clip_state(0))

    def enc(px, ids, mask):
        with torch.no_grad():
            pix = M.clip_preprocess(torch.as_tensor(np.ascontiguousarray(px)))
            ie = M.l2n(M.clip_image_features(clip, pix))
            te = M.l2n(M.clip_text_features(clip, torch.as_tensor(ids), torch.as_tensor(mask)))
        return ie, te
    return enc


def _build(tmp, table, rank=0, world=1, out="db.pkl"):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from tables import TableClipProcessor
    from mmf_amd.vault_builder import generate_embeddings_database
    return generate_embeddings_database("clip_detective_best.pth", os.path.join(tmp, "seed.json"),
                                        os.path.join(tmp, out), processor=TableClipProcessor(table),
                                        encode=_oracle_encoder(), val_accuracy=0.75, batch=4,
                                        rank=rank, world=world)


def _worker(rank, world, port, tmp, table):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    db = _build(tmp, table, rank, world, out="db_w2.pkl")
    with open(os.path.join(tmp, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump({"img": db["image_embeddings"], "ids": db["article_ids"]}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_vault_builder_schema_and_sharded_allgather(tmp_path, capsys):
    tmp = str(tmp_path)
    torch.set_num_threads(4)
    arts, table = _articles(tmp)
    db = _build(tmp, table)
    assert "Error processing id4" in capsys.readouterr().out
    keep = [a for i, a in enumerate(arts) if i != 4]
    with open(os.path.join(tmp, "db.pkl"), "rb") as f:
        disk = pickle.load(f)  # our own file
    assert set(disk) == {"article_ids", "text_contents", "image_paths", "image_embeddings", "text_embeddings",
                         "metadata"}
    assert disk["article_ids"] == [a["article_id"] for a in keep]
    assert disk["text_contents"] == [a["text_content"] for a in keep]
    assert disk["image_paths"] == [a["image_local_path"] for a in keep]
    assert disk["image_embeddings"].shape == (8, 512) and disk["text_embeddings"].shape == (8, 512)
    # model_path is made absolute like train_clip_detective.py:476-477 does
    assert disk["metadata"] == {"model_path": os.path.join(os.getcwd(), "clip_detective_best.pth"),
                                "total_articles": 9, "embedding_dim": 512, "val_accuracy": 0.75}
    np.testing.assert_allclose(np.linalg.norm(disk["image_embeddings"], axis=1), 1.0, atol=1e-5)
    with open(os.path.join(tmp, "db_summary.json")) as f:
        s = json.load(f)
    assert s["total_articles"] == 8 and s["embedding_dimension"] == 512 and s["sample_articles"] == [
        a["article_id"] for a in keep[:5]]
    # reference-order single-article encoding (train_clip_detective.py:533-566 loop)
    enc = _oracle_encoder()
    from mmf_amd import io_utils
    one = []
    for a in keep:
        px = io_utils.clip_pixels(io_utils.to_pil(a["image_local_path"]))[None]
        ids = np.asarray([table[a["text_content"]]], np.int32)
        ie, te = enc(px, ids, np.ones_like(ids))
        one.append(ie[0].numpy())
    np.testing.assert_allclose(disk["image_embeddings"], np.stack(one), atol=2e-5)
    # the vault reader of the analyze path accepts the file (misinfo_forensics.py:222-246 format 2)
    emb, meta = io_utils.load_vault(os.path.join(tmp, "db.pkl"))
    assert emb.shape == (8, 512) and meta[0]["title"] == keep[0]["text_content"]
    # world-size-2 gloo: shards of 5 + 4 articles, one all-gather -> the same database
    mp.start_processes(_worker, args=(2, _free_port(), tmp, table), nprocs=2, join=True, start_method="spawn")
    with open(os.path.join(tmp, "db_w2.pkl"), "rb") as f:
        w2 = pickle.load(f)
    assert w2["article_ids"] == disk["article_ids"]
    np.testing.assert_allclose(w2["image_embeddings"], disk["image_embeddings"], atol=2e-5)
    np.testing.assert_allclose(w2["text_embeddings"], disk["text_embeddings"], atol=2e-5)
    for r in (0, 1):  # every rank holds the full replicated table after the all-gather
        with open(os.path.join(tmp, f"rank{r}.pkl"), "rb") as f:
            rr = pickle.load(f)
        assert rr["ids"] == disk["article_ids"] and rr["img"].shape == (8, 512)
