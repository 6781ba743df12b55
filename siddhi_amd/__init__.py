"""siddhi_amd — MI355X-native pattern/sequence matcher for Siddhi's CEP state engine.

The product path is the HIP engine in siddhi_amd/csrc behind the C-ABI declared in
include/siddhi_gpu.h; siddhi_amd.runtime mirrors Siddhi's host API (SiddhiManager,
SiddhiAppRuntime, InputHandler, QueryCallback, StreamCallback) on top of it.
"""
from .runtime import (CannotRestoreSiddhiAppStateException, Event, InMemoryPersistenceStore,  # noqa: F401
                      InputHandler, NoPersistenceStoreException, PersistenceStore, QueryCallback,
                      SiddhiAppCreationException, SiddhiAppRuntime, SiddhiManager, StreamCallback)
