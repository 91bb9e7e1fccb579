"""Which schedule lets the C5 test's 6-layer model (utils.pipeline.Pipeline,
6 images, one shared caption, seed 61) memorise its caption? Loss every 200
steps per schedule.
  python tools/probes/train_c5.py"""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def run(name, lr, steps=1600, n_img=6, seed=61, T=32, vocab=10000):
    import fpnmt
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from utils.pipeline import Pipeline
    from test_gpu_configs import _images
    fpnmt.set_precision("bf16")
    pl = Pipeline(max_seq_len=T, target_vocab_size=vocab, image_size=224, n_layers=6, rate=0.0,
                  init=Init(torch.Generator().manual_seed(seed)), use_graph=False)
    imgs = _images(n_img, 224, seed=seed + 1)
    g = torch.Generator().manual_seed(seed + 2)
    tok = torch.zeros(n_img, T, dtype=torch.int64)
    cap = torch.randint(4, vocab, (T - 3,), generator=g)
    tok[:, 0] = pl.start_token
    tok[:, 1:T - 2] = cap
    tok[:, T - 2] = pl.end_token
    eng = TrainEngine(pl.transformer, lr, use_graph=True)
    di, dt = imgs.cuda(), tok.cuda()
    t0 = time.time()
    out = []
    for i in range(steps):
        loss = eng.step(di, dt)
        if i % 200 == 0 or i == steps - 1:
            out.append(round(float(loss), 3))
    print(f"{name:34s}: {out} ({time.time() - t0:.1f} s)", flush=True)
    del eng, pl
    torch.cuda.empty_cache()
    fpnmt.layers.invalidate_weights()


def main():
    from utils.utils import CustomSchedule
    run("const 1e-4", 1e-4)
    run("const 5e-5", 5e-5)
    run("const 2e-5", 2e-5)
    run("warm-up 400 -> 1e-4 (d=156250)", CustomSchedule(156250, 400))
    run("warm-up 400 -> 2e-4 (d=39062)", CustomSchedule(39062, 400))


if __name__ == "__main__":
    main()
