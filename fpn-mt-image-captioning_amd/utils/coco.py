"""COCO caption annotations: the subset of pycocotools.coco.COCO the
reference's data side calls (dataset.py:45-51,85,175-186,212-240,275-321):
getAnnIds, getImgIds, loadAnns, loadImgs, loadRes, showAnns, imgToAnns.
pycocotools is not installed here, so this restates its
behaviour for caption files (`captions_<split>.json`: images + annotations
with image_id / caption).
"""
from __future__ import annotations

import copy
import json
from collections import defaultdict


def _as_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple, set)) else [x]


class COCO:
    def __init__(self, annotation_file=None):
        self.dataset = {}
        self.anns, self.imgs, self.cats = {}, {}, {}
        self.imgToAnns = defaultdict(list)
        if annotation_file is not None:
            with open(annotation_file) as f:
                dataset = json.load(f)
            if not isinstance(dataset, dict):
                raise ValueError(f"annotation file format {type(dataset)} not supported")
            self.dataset = dataset
            self.createIndex()

    def createIndex(self):
        anns, imgs, cats = {}, {}, {}
        img_to_anns = defaultdict(list)
        for ann in self.dataset.get("annotations", []):
            img_to_anns[ann["image_id"]].append(ann)
            anns[ann["id"]] = ann
        for img in self.dataset.get("images", []):
            imgs[img["id"]] = img
        for cat in self.dataset.get("categories", []):
            cats[cat["id"]] = cat
        self.anns, self.imgs, self.cats, self.imgToAnns = anns, imgs, cats, img_to_anns

    def getAnnIds(self, imgIds=(), catIds=(), areaRng=(), iscrowd=None):
        img_ids = _as_list(imgIds)
        if not img_ids:
            anns = self.dataset.get("annotations", [])
        else:
            anns = [a for i in img_ids if i in self.imgToAnns for a in self.imgToAnns[i]]
        return [a["id"] for a in anns]

    def getImgIds(self, imgIds=(), catIds=()):
        img_ids = _as_list(imgIds)
        return list(set(img_ids)) if img_ids else list(self.imgs.keys())

    def loadAnns(self, ids=()):
        if isinstance(ids, (list, tuple)):
            return [self.anns[i] for i in ids]
        return [self.anns[ids]]

    def loadImgs(self, ids=()):
        if isinstance(ids, (list, tuple)):
            return [self.imgs[i] for i in ids]
        return [self.imgs[ids]]

    def loadRes(self, resFile):
        """Result captions [{'image_id', 'caption'}] as a COCO object
        (ids 1..n in file order, images restricted to the captioned ones)."""
        res = COCO()
        res.dataset["images"] = [img for img in self.dataset.get("images", [])]
        if isinstance(resFile, str):
            with open(resFile) as f:
                anns = json.load(f)
        else:
            anns = copy.deepcopy(resFile)
        if not isinstance(anns, list):
            raise AssertionError("results in not an array of objects")
        ann_img_ids = {a["image_id"] for a in anns}
        if not ann_img_ids <= set(self.getImgIds()):
            raise AssertionError("Results do not correspond to current coco set")
        if anns and "caption" in anns[0]:
            keep = {img["id"] for img in res.dataset["images"]} & ann_img_ids
            res.dataset["images"] = [img for img in res.dataset["images"] if img["id"] in keep]
            for i, ann in enumerate(anns):
                ann["id"] = i + 1
        res.dataset["annotations"] = anns
        res.createIndex()
        return res

    def showAnns(self, anns):
        for ann in anns:
            print(ann["caption"])
