"""Table-driven tokenizers (text string -> pre-generated token ids) used wherever the real vocab
files are unavailable: by make_golden.py to drive the reference, and by the API parity tests to
drive the drop-in API with the same ids."""
import torch
from transformers import BatchEncoding, CLIPImageProcessor


class TableRobertaTokenizer:
    def __init__(self, table):
        self.table = table

    def __call__(self, text, return_tensors="pt", max_length=512, truncation=True, padding=True):
        texts = [text] if isinstance(text, str) else list(text)
        seqs = [list(self.table[s])[:max_length] if truncation else list(self.table[s]) for s in texts]
        L = max(len(s) for s in seqs)
        ids = torch.full((len(seqs), L), 1, dtype=torch.long)  # RoBERTa pad id, right padding
        mask = torch.zeros((len(seqs), L), dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.tensor(s)
            mask[i, :len(s)] = 1
        return BatchEncoding({"input_ids": ids, "attention_mask": mask})


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
