"""Table-driven tokenizers (text string -> pre-generated token ids) used wherever the real vocab
files are unavailable: by make_golden.py to drive the reference, and by the API parity tests to
drive the drop-in API with the same ids."""
import torch
from transformers import BatchEncoding, CLIPImageProcessor


class TableRobertaTokenizer:
    def __init__(self, table):
        self.table = table

    def __call__(self, text, return_tensors="pt", max_length=512, truncation=True, padding=True):
        ids = list(self.table[text])[:max_length] if truncation else list(self.table[text])
        t = torch.tensor([ids], dtype=torch.long)
        return BatchEncoding({"input_ids": t, "attention_mask": torch.ones_like(t)})


class TableClipProcessor:
    def __init__(self, table, eos_id: int = 49407):
        self.table = table
        self.eos_id = eos_id
        self.image_processor = CLIPImageProcessor()

    def __call__(self, text=None, images=None, return_tensors="pt", padding=False, truncation=False):
        out = {}
        if text is not None:
            seqs = [list(self.table[s]) for s in text]
            if truncation:
                seqs = [s[:77] for s in seqs]
            L = max(len(s) for s in seqs)
            ids = torch.full((len(seqs), L), self.eos_id, dtype=torch.long)
            mask = torch.zeros((len(seqs), L), dtype=torch.long)
            for i, s in enumerate(seqs):
                ids[i, :len(s)] = torch.tensor(s)
                mask[i, :len(s)] = 1
            out["input_ids"], out["attention_mask"] = ids, mask
        if images is not None:
            out["pixel_values"] = self.image_processor(images=images, return_tensors="pt")["pixel_values"]
        return BatchEncoding(out)
