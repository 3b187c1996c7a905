"""Drop-in for the reference's evaluation CLI (test.py:61-83, :168-344) for --model raa:

    python test.py --dataset sbmrgbd --model raa --gpus 0 [--checkpoint snapshot.pth]

For every target frame: the mean over `sample_range` reference frames of the model's x1
(test.py:287-305), resized to output_WH with bilinear half-pixel interpolation (cv2.resize
INTER_LINEAR, :309-314), quantised (output * 255).astype(uint8) (:317), scored with the soft
IoU of evaluation.py:3-22 (:321), logged as "##== seq: S frame: F IOU: J==##" (:322) and saved
as a PNG mask (:332-340); the run ends with "##== final IOU: mean==##" (:342-344).

MI355X-native: the N references run as ONE batched forward with the target encoded once
(cosnet_amd.inference.multi_reference_x1; equal to the reference's loop in eval mode), the
average and the resize are HIP kernels; only the uint8 masks cross to the host.  Checkpoints
load with torch.load(weights_only=True); "module." prefixes are stripped (test.py:140-161).
`--dataset sbmrgbd` reads the SBM-RGBD tree (cosnet_amd/sbm_rgbd.py, GPU frame preparation);
`--dataset synthetic` evaluates seeded frame pairs (cosnet_amd/data.py).
"""
import argparse
import datetime
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

LOG_START, LOG_END = "##==", "==##"


def get_arguments(argv=None):
    p = argparse.ArgumentParser(description="RGBDCoAttention")
    p.add_argument("--dataset", type=str, default="synthetic")
    p.add_argument("--cuda", default=True)
    p.add_argument("--gpus", type=str, default="0")
    p.add_argument("--seq_name", default="bmx-bumps")
    p.add_argument("--use_crf", default="True")
    p.add_argument("--save_seg_img", default="True")
    p.add_argument("--sample_range", default=5)
    p.add_argument("--epoches", default=0)
    p.add_argument("--batch_size", default=0)
    p.add_argument("--model", default="raa")
    # this build
    p.add_argument("--config", default=os.path.join(REPO, "config.yaml"))
    p.add_argument("--checkpoint", default=None, help="overrides test.model.<name>.pretrained_params")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                   help="bf16 (default): the MI355X throughput path, fused co-attention; fp32: the reference arithmetic")
    p.add_argument("--result-root", default=".")
    p.add_argument("--frames", type=int, default=None, help="synthetic: number of target frames")
    return p.parse_args(argv)


def config(args, user_config):
    """test.py:86-137 (sbmrgbd / synthetic)."""
    ds = user_config["test"]["dataset"].get(args.dataset)
    if ds is None:
        raise SystemExit("dataset error: %r" % args.dataset)
    args.batch_size = int(args.batch_size) if args.batch_size else 1
    args.epoches = int(args.epoches) if args.epoches else 15
    args.num_classes = 2
    args.data_path = ds.get("data_path", "")
    args.sample_range = int(ds["sample_range"])  # the YAML overrides the flag (test.py:132)
    h, w = map(int, str(ds["image_HW_4_model"]).split(","))
    args.image_HW_4_model = (h, w)
    w, h = map(int, str(ds["output_WH"]).split(","))
    args.output_WH = (w, h)
    args.frames = args.frames if args.frames is not None else int(ds.get("frames", 8))
    args.subset = ds.get("subset") or None


def main(argv=None):
    args = get_arguments(argv)
    os.environ["CUDA_VISIBLE_DEVICES"] = args.gpus  # test.py:175, before HIP starts
    import numpy as np
    import torch
    import yaml

    import cosnet_amd as C
    from cosnet_amd.checkpoint import convert_state_dict, load_checkpoint
    from cosnet_amd.data import SyntheticRGBDPairs
    from cosnet_amd.inference import multi_reference_x1, resize_linear, soft_iou

    with open(args.config) as f:
        user_config = yaml.safe_load(f)
    config(args, user_config)
    if args.model not in ("raa", "resnet_aspp_add"):
        print("Invalid model name!")
        return 1
    args.full_model_name = "resnet_aspp_add"
    if not torch.cuda.is_available():
        raise Exception("No GPU found or Wrong gpu id, please run without --cuda")
    dev = torch.device("cuda:0")
    stamp = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
    args.result_dir = os.path.join(args.result_root, "vos_test_results", args.dataset,
                                   args.full_model_name, stamp)
    os.makedirs(args.result_dir, exist_ok=True)
    log_name = os.path.join(args.result_dir, "%s__%s_%s_test_log.txt" % (args.dataset, args.full_model_name, stamp))
    logger = open(log_name, "a")
    ckpt = args.checkpoint or user_config["test"]["model"][args.full_model_name].get("pretrained_params", "")
    args.pretrained_params = ckpt
    logger.write(LOG_START + str(args) + LOG_END + "\n")
    logger.flush()

    model = C.build_model(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    if ckpt:
        model.load_state_dict(convert_state_dict(load_checkpoint(ckpt)["model"]))
    else:
        print("no pretrained_params given: seeded initialisation (scores are meaningless)")
    model.eval()
    model.to(dev)

    if args.dataset == "sbmrgbd":
        from cosnet_amd.sbm_rgbd import SBMRGBD
        if not args.data_path or not os.path.isdir(args.data_path):
            raise SystemExit("sbmrgbd: data_path %r not found (config.yaml test.dataset.sbmrgbd)" % args.data_path)
        sbm = SBMRGBD(args.data_path, args.sample_range, args.image_HW_4_model, for_training=False,
                      batch_size=args.batch_size, subset_percentage=1, subset=args.subset or None,
                      device=dev)  # test.py:271-272
        db = [sbm.collate([sbm[j] for j in range(i, i + args.batch_size)])
              for i in range(0, len(sbm), args.batch_size)]
    elif args.dataset == "synthetic":
        db = SyntheticRGBDPairs(args.frames // args.batch_size, args.image_HW_4_model, args.batch_size,
                                sample_range=args.sample_range, seed=4321)
    else:
        raise SystemExit("dataset %r: only sbmrgbd and synthetic are provided by this build" % args.dataset)
    out_dir = None
    if str(args.save_seg_img) not in ("False", "0", ""):
        out_dir = os.path.join(args.result_dir, "obj_seg_imgs")
        os.makedirs(out_dir, exist_ok=True)
    out_hw = (args.output_WH[1], args.output_WH[0])
    iou_sum, iou_n = 0.0, 0
    for index, batch in enumerate(db):
        print("%d processd" % index)
        for j in range(args.batch_size):
            tgt = batch["target"][j:j + 1].to(dev)
            tdep = batch["target_depth"][j:j + 1].to(dev)
            srch = torch.cat([batch["search_%d" % i][j:j + 1] for i in range(args.sample_range)]).to(dev)
            sdep = torch.cat([batch["search_%d_depth" % i][j:j + 1] for i in range(args.sample_range)]).to(dev)
            x1 = multi_reference_x1(model, tgt, tdep, srch, sdep)          # [1,1,h,w]
            gt = batch["target_gt"][j:j + 1].unsqueeze(1).float()
            if tuple(gt.shape[2:]) != out_hw:
                gt = torch.nn.functional.interpolate(gt, size=out_hw, mode="nearest")
            # uint8 quantisation (:317) + soft-J (evaluation.py:3-22) in one HIP kernel
            masks, ious, _ = soft_iou(resize_linear(x1, out_hw), gt[:, 0].to(torch.uint8).to(dev))
            mask = masks[0].cpu().numpy()                                  # [H,W] uint8
            iou = float(ious[0].item())
            seq, frame = batch["seq_name"][j], batch["frame_index"][j]
            logger.write(LOG_START + " seq: " + seq + " frame: " + frame + " IOU: " + str(iou) + LOG_END + "\n")
            iou_sum += iou
            iou_n += 1
            if out_dir:
                from PIL import Image
                d = os.path.join(out_dir, seq)
                os.makedirs(d, exist_ok=True)
                Image.fromarray(mask).save(os.path.join(d, "%s.png" % frame))
    final = iou_sum / max(iou_n, 1)
    logger.write(LOG_START + " final IOU: " + str(final) + LOG_END + "\n")
    logger.close()
    print("final IOU: %.6f over %d frames (log: %s)" % (final, iou_n, log_name))
    return 0


if __name__ == "__main__":
    sys.exit(main())
