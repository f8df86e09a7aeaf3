"""Which dtype does the reference's Truth-Vault builder store?  train_clip_detective.py:550-553
encodes under CUDA autocast() and keeps `outputs.image_embeds.cpu().numpy()[0]`; CLIPModel.forward
normalises the fp16 projection output with a norm (transformers 5.x: pow/sum/pow, 4.x: .norm) that
autocast runs in fp32, and fp16 / fp32 promotes to fp32.  Run on the GPU box (needs CUDA autocast):

    python tools/autocast_vault_dtype.py
"""
import json

import torch
from transformers import CLIPConfig, CLIPModel

torch.manual_seed(0)
m = CLIPModel(CLIPConfig()).cuda().eval()
px = torch.randn(2, 3, 224, 224, device="cuda")
ids = torch.randint(0, 49406, (2, 12), device="cuda")
ids[:, -1] = 49407
with torch.no_grad(), torch.cuda.amp.autocast():
    out = m(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), return_dict=True)
    proj = m.visual_projection(m.vision_model(pixel_values=px).pooler_output)
    legacy = proj / proj.norm(p=2, dim=-1, keepdim=True)  # transformers 4.x CLIPModel.forward
res = {"image_embeds": str(out.image_embeds.dtype), "text_embeds": str(out.text_embeds.dtype),
       "projection_output": str(proj.dtype), "legacy_4x_normalised": str(legacy.dtype),
       "numpy_after_cpu": str(out.image_embeds.cpu().numpy().dtype)}
print(json.dumps(res))
