"""SMPL skeleton tree (SkeletonTree.from_mjcf, puffer_phc/poselib_skeleton.py:275-320).

The packaged table `assets/smpl_skeleton.json` holds the 24 node names, parent indices and
local translations of the SMPL humanoid MJCF in DFS order; `from_mjcf` parses any MJCF the
same way for users who bring their own asset.
"""

import json
import os
import xml.etree.ElementTree as ET

import numpy as np
import torch

_ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "smpl_skeleton.json")


class SkeletonTree:
    def __init__(self, node_names, parent_indices, local_translation):
        if not (len(node_names) == len(parent_indices) == len(local_translation)):
            raise ValueError("node_names, parent_indices and local_translation must have equal length")
        self.node_names = list(node_names)
        self.parent_indices = torch.as_tensor(np.asarray(parent_indices), dtype=torch.long)
        self.local_translation = torch.as_tensor(np.asarray(local_translation, dtype=np.float32))

    def __len__(self):
        return len(self.node_names)

    @property
    def num_joints(self):
        return len(self)

    def index(self, name):
        return self.node_names.index(name)

    @classmethod
    def from_mjcf(cls, path):
        root = ET.parse(path).getroot()
        world = root.find("worldbody")
        if world is None or world.find("body") is None:
            raise ValueError("MJCF parsed incorrectly please verify it.")
        names, parents, offsets = [], [], []

        def visit(node, parent):
            idx = len(names)
            names.append(node.attrib.get("name"))
            parents.append(parent)
            offsets.append(np.array(node.attrib.get("pos", "0 0 0").split(), dtype=np.float64))
            for child in node.findall("body"):
                visit(child, idx)

        visit(world.find("body"), -1)
        return cls(names, np.array(parents, np.int64), np.stack(offsets).astype(np.float32))

    @classmethod
    def smpl(cls):
        with open(_ASSET) as f:
            d = json.load(f)
        return cls(d["node_names"], d["parent_indices"], np.array(d["local_translation"], np.float32))
