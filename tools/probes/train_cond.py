"""Image-conditioned memorisation (VERDICT r04 'next' #1): can the decode
parity fixtures' models learn ONE DISTINCT caption per image, so that the
decoded ids depend on the image? Per setting: the training loss curve, the
pairwise cosine of the images' encoder outputs (how far apart the images look
to the model), and the GPU greedy decode of every image against its own
caption.
  python tools/probes/train_cond.py [quick]"""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def run(name, layers, vocab, n_img, lr, steps, seed, kind, T=32):
    import fpnmt
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from utils.pipeline import Pipeline
    from test_gpu_configs import _images, _structured_images
    fpnmt.set_precision("bf16")
    pl = Pipeline(max_seq_len=T, target_vocab_size=vocab, image_size=224, n_layers=layers, rate=0.0,
                  init=Init(torch.Generator().manual_seed(seed)), use_graph=False)
    imgs = (_structured_images if kind == "structured" else _images)(n_img, 224, seed=seed + 1)
    g = torch.Generator().manual_seed(seed + 2)
    tok = torch.zeros(n_img, T, dtype=torch.int64)
    for i in range(n_img):
        tok[i, 0] = pl.start_token
        tok[i, 1:T - 2] = torch.randint(4, vocab, (T - 3,), generator=g)
        tok[i, T - 2] = pl.end_token
    eng = TrainEngine(pl.transformer, lr, use_graph=True)
    di, dt = imgs.cuda(), tok.cuda()
    t0 = time.time()
    curve = []
    for i in range(steps):
        loss = eng.step(di, dt)
        if i % 200 == 0 or i == steps - 1:
            curve.append(round(float(loss), 3))
    fpnmt.set_precision("fp32")
    with torch.no_grad():
        enc = pl.transformer.encoder(di, False, None).float().reshape(n_img, -1)
        en = enc / enc.norm(dim=1, keepdim=True)
        cos = (en @ en.T)
        off = cos[~torch.eye(n_img, dtype=torch.bool, device=cos.device)]
    mem = []
    for i in range(n_img):
        ids = pl.predict(imgs[i].cuda(), T)[0].cpu().tolist()
        target = [int(t) for t in tok[i, 1:] if int(t) not in (0, pl.end_token)]
        mem.append(ids == target)
    print(f"{name:44s}: loss {curve} | enc cos off-diag max {float(off.max()):.4f} mean {float(off.mean()):.4f} | "
          f"memorised {sum(mem)}/{n_img} {mem} ({time.time() - t0:.1f} s)", flush=True)
    del eng, pl
    torch.cuda.empty_cache()
    fpnmt.layers.invalidate_weights()


def main():
    from utils.utils import CustomSchedule
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    if len(sys.argv) > 1 and sys.argv[1] == "2L":
        for seed in (61, 71, 81, 91):
            for steps in (300, 800):
                run(f"2L V1000 4 img structured seed {seed} const 3e-4 {steps}", 2, 1000, 4, 3e-4, steps, seed,
                    "structured")
        run("2L V1000 4 img structured seed 71 warm400->1e-4 1600", 2, 1000, 4, CustomSchedule(156250, 400), 1600,
            71, "structured")
        run("2L V1000 6 img structured seed 71 const 1e-4 1200", 2, 1000, 6, 1e-4, 1200, 71, "structured")
        return
    run("2L V1000 4 img noise const 3e-4 300", 2, 1000, 4, 3e-4, 300, 71, "noise")
    run("2L V1000 4 img structured const 3e-4 300", 2, 1000, 4, 3e-4, 300, 71, "structured")
    run("2L V1000 4 img structured const 3e-4 800", 2, 1000, 4, 3e-4, 800, 71, "structured")
    if quick:
        return
    run("6L V10k 6 img structured warm400->1e-4 1600", 6, 10000, 6, CustomSchedule(156250, 400), 1600, 61,
        "structured")
    run("6L V10k 6 img structured warm400->1e-4 3000", 6, 10000, 6, CustomSchedule(156250, 400), 3000, 61,
        "structured")


if __name__ == "__main__":
    main()
