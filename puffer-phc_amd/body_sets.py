"""SMPL body/DOF name sets (puffer_phc/body_sets.py:11-71) and index helpers."""

BODY_NAMES = (
    "Pelvis", "L_Hip", "L_Knee", "L_Ankle", "L_Toe", "R_Hip", "R_Knee", "R_Ankle", "R_Toe",
    "Torso", "Spine", "Chest", "Neck", "Head", "L_Thorax", "L_Shoulder", "L_Elbow", "L_Wrist",
    "L_Hand", "R_Thorax", "R_Shoulder", "R_Elbow", "R_Wrist", "R_Hand",
)
DOF_NAMES = BODY_NAMES[1:]
REMOVE_NAMES = ("L_Hand", "R_Hand", "L_Toe", "R_Toe")
KEY_BODIES = ("R_Ankle", "L_Ankle", "R_Wrist", "L_Wrist")
CONTACT_BODIES = ("R_Ankle", "L_Ankle", "R_Toe", "L_Toe")
TRACK_BODIES = BODY_NAMES
RESET_BODIES = TRACK_BODIES
EVAL_BODIES = tuple(name for name in BODY_NAMES if name not in REMOVE_NAMES)
JOINT_GROUPS = [
    ["L_Hip", "L_Knee", "L_Ankle", "L_Toe"],
    ["R_Hip", "R_Knee", "R_Ankle", "R_Toe"],
    ["Pelvis", "Torso", "Spine", "Chest", "Neck", "Head"],
    ["L_Thorax", "L_Shoulder", "L_Elbow", "L_Wrist", "L_Hand"],
    ["R_Thorax", "R_Shoulder", "R_Elbow", "R_Wrist", "R_Hand"],
]
LIMB_WEIGHT_GROUP = [[BODY_NAMES.index(j) for j in g] for g in JOINT_GROUPS]


def body_ids(names, targets=BODY_NAMES):
    return [names.index(t) for t in targets]


def build_body_ids_tensor(body_names, target_names, device):
    import torch

    return torch.tensor([body_names.index(n) for n in target_names], device=device, dtype=torch.long)


def dof_subset():
    """Indices of the 19 AMP joints' dofs (humanoid_phc.py:185-194)."""
    out = []
    for i, name in enumerate(DOF_NAMES):
        if name not in REMOVE_NAMES:
            out.extend(range(3 * i, 3 * i + 3))
    return out
