"""client"""
