"""The `core/hardware_accel.py` names this build replaces.

The reference module picks an onnxruntime execution provider and creates sessions for every
stage (`core/hardware_accel.py:206-697`).  ASR no longer uses onnxruntime (it runs in
libzasr.so), and per the north star the DirectML / OpenVINO add-on DLL dispatch is removed.

zasr.dropin.install(..., accel_module=core.hardware_accel) rebinds:

  configure_gpu_addon_paths  no add-on directories (the dispatch is removed)
  create_ort_session         the two config-5 stages this build runs on the GPU are served by
                             libzasr.so sessions with the onnxruntime `run` surface their
                             callers use -- "CAM++ speaker embedding"
                             (core/speaker_diarization_senko_campp_optimized.py:364-368, run at
                             :381 and :604: run(['embs'], {'feats': [N, T, 80]})) and "ViBERT
                             punctuation" (core/gec_model.py:168-172, run at :387 / :397:
                             run(None, feeds) -> [logits, detect_logits]); every other stage
                             (pyannote, DNSMOS, ...) goes to the reference's own function
  is_gpu_provider            also true for ZASR_PROVIDER, so the callers' GPU checks
                             (core/gec_model.py:173, :189) keep the session
  auto_batch_size            for ZASR_PROVIDER: the launch groups measured best on MI355X
                             (CAM++ 4096 windows; ViBERT 128 rows: its results
                             are the same at any mini-batch size); otherwise the reference's

The reference's callers reach create_ort_session only when their execution provider policy
is not "cpu" (config `execution_provider` or `ASR_VN_ACCEL`, core/asr_engine.py:1980-1983;
core/speaker_diarization_senko_campp_optimized.py:363; core/gec_model.py:123-126): with
"cpu" they build onnxruntime CPU sessions directly, as the user asked.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Tuple

ZASR_PROVIDER = "ZasrMI355XExecutionProvider"
CAMPP_BATCH = 4096
VIBERT_BATCH = 128


def configure_gpu_addon_paths() -> List[str]:
    """The reference adds the DirectML / OpenVINO / CUDA add-on directories to the DLL search
    path and returns them (`core/hardware_accel.py:60-118`); that dispatch is removed, so there
    are none."""
    return []


def stage_kind(model_path: str, stage: str) -> Optional[str]:
    """Which libzasr.so engine serves a create_ort_session call: the reference's own stage
    labels and file names (the CAM++ test of core/hardware_accel.py:567-571; ViBERT's
    stage label at core/gec_model.py:171 and file names at :133-134)."""
    s = str(stage or "").lower()
    m = os.path.basename(str(model_path or "")).lower()
    if "cam++" in s or "campp" in s or "campplus" in m:
        return "campp"
    if "vibert" in s or "punct" in s or m.startswith("vibert-capu"):
        return "vibert"
    return None


def _device_id() -> int:
    return int(os.environ.get("ZASR_DEVICE", os.environ.get("LOCAL_RANK", "0")) or 0)


class CamppOrtSession:
    """CAM++ on the GPU behind the onnxruntime surface the diarizer calls:
    run(['embs'] or None, {'feats': f32[N, T, 80]}) -> [f32[N, 192]]."""

    def __init__(self, model_path: str, device_id: int = 0):
        from zasr.binding import CamppEmbedder
        self.model_path = model_path
        self.engine = CamppEmbedder(model_path, device_id)

    def run(self, output_names, feeds: Dict[str, Any]):
        if output_names not in (None, ["embs"], ("embs",)):
            raise KeyError(f"CAM++ session has one output 'embs', asked {output_names}")
        return [self.engine.embed(feeds["feats"])]

    def get_providers(self) -> List[str]:
        return [ZASR_PROVIDER]


class VibertOrtSession:
    """ViBERT-capu on the GPU behind the onnxruntime surface GecBERTModel calls:
    run(None, {input_ids, attention_mask, token_type_ids, input_offsets}) ->
    [logits, detect_logits] (zasr.binding.VibertSession)."""

    def __init__(self, model_path: str, device_id: int = 0):
        from zasr.binding import VibertSession
        self.model_path = model_path
        self.engine = VibertSession(model_path, device_id)

    def run(self, output_names, feeds: Dict[str, Any]):
        return self.engine.run(output_names, feeds)

    def get_providers(self) -> List[str]:
        return [ZASR_PROVIDER]


def make_create_ort_session(orig: Callable) -> Callable:
    """The rebound create_ort_session: same signature and (session, info) return as the
    reference's (core/hardware_accel.py:555-621); CAM++ and ViBERT get libzasr.so sessions
    (no onnxruntime session is built for them), every other stage the reference's function."""

    def create_ort_session(ort_module: Any, model_path: str, sess_options: Any,
                           policy: str = "cpu", stage: str = "") -> Tuple[Any, Dict[str, Any]]:
        kind = stage_kind(model_path, stage)
        if kind is None:
            return orig(ort_module, model_path, sess_options, policy=policy, stage=stage)
        sess = (CamppOrtSession if kind == "campp" else VibertOrtSession)(model_path, _device_id())
        info = {"stage": stage, "policy": policy, "requested_providers": [ZASR_PROVIDER],
                "actual_provider": ZASR_PROVIDER, "session_providers": [ZASR_PROVIDER],
                "used_gpu": True, "fallback_reason": None,
                "engine": f"libzasr.so {kind} (HIP, gfx950)", "model_path": model_path}
        return sess, info

    create_ort_session._zasr_wrapped = True
    create_ort_session.__doc__ = getattr(orig, "__doc__", None)
    return create_ort_session


def make_is_gpu_provider(orig: Callable) -> Callable:
    def is_gpu_provider(provider: Optional[str]) -> bool:
        return provider == ZASR_PROVIDER or orig(provider)

    is_gpu_provider._zasr_wrapped = True
    return is_gpu_provider


def make_auto_batch_size(orig: Callable) -> Callable:
    def auto_batch_size(stage: str, default: int, provider: Optional[str] = None) -> int:
        if provider == ZASR_PROVIDER:
            kind = stage_kind("", stage)
            if kind == "campp":
                return CAMPP_BATCH
            if kind == "vibert":
                return VIBERT_BATCH
            return int(default)
        return orig(stage, default, provider)

    auto_batch_size._zasr_wrapped = True
    return auto_batch_size
